"""Out-of-core read of a BAM larger than one GPU's HBM ("Streaming").

A file on one GPU needs C + U + SoA bytes of HBM (about 1 + 2.85 + 0.53 x its compressed size for
short reads), so a 100 GB 30x-WGS BAM (configs[2]) does not fit a 288 GB MI355X at once.  It is
read in windows: consecutive groups of whole Disq partitions of about `window` compressed bytes,
each decoded as a shard (its own bytes plus the halo that holds its last partition's straddling
record, dq_open_shard) -- the single-GPU form of the multi-GPU byte-range shards.  `depth`
contexts, each with its own HIP stream and buffers, work on successive windows from their own
host threads, so the host read and H2D copy of one window overlap the kernels of another.

The result is the same per-partition record counts and digests, in partition order, as the
whole-file run: the window boundaries are partition boundaries, and a shard reproduces the
partitions it owns bit for bit (tests/test_parallel.py, tests/test_stream.py).
"""
from __future__ import annotations

import math
import threading
import time
from typing import Optional

import numpy as np

from . import parallel as P


def stream_read(read_bytes, file_len: int, header: bytes,
                window: int = 8 << 30, depth: int = 2, split_size: int = 0,
                use_nio: bool = False, hadoop_block_size: int = 0, device: int = 0,
                verify_crc: bool = True, halo: int = 4 << 20, on_window=None,
                contexts=None, ramp: bool = False) -> dict:
    """Decode the whole file in windows of ~`window` compressed bytes on one GPU.

    read_bytes(a, b) returns the file's bytes [a, b) (page cache, host memory or a generator), or
    read_bytes is a path: the library reads each window itself (dq_open_shard_path).
    on_window(k, ctx, shard), if given, runs on the window's context after its pipeline (e.g. to
    export records with ctx.read()).  contexts: `depth` open Contexts to use (e.g. set up with an
    export arena beforehand); they stay open.  ramp: smaller first and last windows (the pipeline's
    fill and drain).  Returns the per-partition counts and digests, the
    whole-file digest, record and decompressed byte totals, and timings."""
    from . import _lib
    split_opts = dict(split_size=split_size, use_nio=use_nio, hadoop_block_size=hadoop_block_size)
    nwin = max(1, math.ceil(file_len / max(1, window)))
    offsets = None
    if ramp and file_len > 2 * window:
        # windows of window/4, window/2, then window, ..., then window/2, window/4: the first
        # export starts after a quarter window's read and pipeline instead of a whole one's, and
        # the last one drains a quarter window's export
        sizes = [window // 4, window // 2]
        tail = [window // 2, window // 4]
        mid = file_len - sum(sizes) - sum(tail)
        nmid = max(1, math.ceil(mid / window))
        sizes += [mid // nmid + (1 if i < mid % nmid else 0) for i in range(nmid)] + tail
        offsets = [0]
        for z in sizes:
            offsets.append(offsets[-1] + z)
        offsets[-1] = file_len
        nwin = len(sizes)
    plan = [s for s in P.shard_plan(file_len, nwin, offsets=offsets, **split_opts) if not s.empty]
    nsplit = len(P.path_splits(file_len, **split_opts))
    counts = np.zeros(nsplit, np.int64)
    digests = np.zeros(nsplit, np.uint64)
    totals = {"records": 0, "owned_bytes": 0, "compressed_read": 0, "ms_device": 0.0,
              "open_s": 0.0, "run_s": 0.0, "on_window_s": 0.0}
    lock = threading.Lock()
    nxt = [0]
    errors = []

    import contextlib

    def worker(slot):
        try:
            cm = (contextlib.nullcontext(contexts[slot]) if contexts is not None else
                  _lib.Context(split_size=split_size, use_nio=use_nio,
                               hadoop_block_size=hadoop_block_size, verify_crc=verify_crc,
                               device=device))
            with cm as c:
                while True:
                    with lock:
                        k = nxt[0]
                        nxt[0] += 1
                    if k >= len(plan) or errors:
                        return
                    s = plan[k]
                    h = halo
                    while True:
                        end = min(file_len, s.hi + h)
                        try:
                            t0 = time.perf_counter()
                            if isinstance(read_bytes, str):
                                c.open_shard_path(read_bytes, s.lo, end - s.lo, s.p0, s.p1, header)
                            else:
                                c.open_shard(read_bytes(s.lo, end), s.lo, file_len, s.p0, s.p1,
                                             header)
                            t1 = time.perf_counter()
                            st = c.run_resident()
                            t2 = time.perf_counter()
                            break
                        except _lib.DqError as e:
                            if "halo too small" in str(e) and end < file_len:
                                h *= 4
                                continue
                            raise
                    cnt, dig = c.partition_digests()
                    t3 = time.perf_counter()
                    if on_window is not None:
                        on_window(k, c, s)
                    t4 = time.perf_counter()
                    with lock:
                        totals["open_s"] += t1 - t0
                        totals["run_s"] += t2 - t1
                        totals["on_window_s"] += t4 - t3
                        counts[s.p0:s.p1] = cnt
                        digests[s.p0:s.p1] = dig
                        totals["records"] += st.n_records
                        totals["owned_bytes"] += st.owned_bytes
                        totals["compressed_read"] += end - s.lo
                        totals["ms_device"] += st.ms_total
        except BaseException as e:  # noqa: BLE001 -- re-raised by the caller's thread
            with lock:
                errors.append(e)

    t0 = time.perf_counter()
    nth = max(1, min(depth if contexts is None else len(contexts), len(plan)))
    th = [threading.Thread(target=worker, args=(i,)) for i in range(nth)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    if errors:
        raise errors[0]
    return {"counts": counts, "digests": digests,
            "digest": P.fold_digest([int(x) for x in digests]),
            "n_records": int(counts.sum()), "windows": len(plan), "seconds": wall, **totals}


def stream_read_path(path: str, header: Optional[bytes] = None, **kw) -> dict:
    """stream_read over a file on disk (or in the page cache)."""
    import os
    file_len = os.path.getsize(path)

    if header is None:
        from . import _lib

        def prefix(n):
            with open(path, "rb") as f:
                return f.read(n)
        with _lib.Context(device=kw.get("device", 0)) as c:
            header = P.broadcast_header(c.header_from_prefix, prefix, file_len, 0, 1)
    return stream_read(path, file_len, header, **kw)
