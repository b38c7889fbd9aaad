"""Dev tool: end-to-end read (page cache -> HBM -> pipeline -> host SoA + raw bytes) of one file,
as bench.py's end_to_end leg, for A/B runs of the upload path and the window/depth settings.

  python tools/e2e_ab.py gen PATH GB          # a configs[2]-shaped file in PATH (e.g. /dev/shm)
  python tools/e2e_ab.py run PATH [--window-gb 2 --depth 3 --reps 2]   # one JSON line per rep
Environment knobs of the library apply per process (DQ_MMAP=0: pinned staging instead of the
registered page-cache mapping).
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def gen(path, gb):
    import numpy as np
    from disq_amd import synth
    probe = synth.generate(20000, seed=1, nthreads=16)
    n = int(gb * 1e9 / (len(probe.bam) / probe.n_records))
    res, free = synth.generate(n, seed=1, nthreads=16, as_buffer=True, unplaced_fraction=0.005)
    buf = np.ctypeslib.as_array((ctypes.c_uint8 * res.bam_len).from_address(res.bam))
    with open(path, "wb") as f:
        f.write(memoryview(buf))
    free()
    print(json.dumps({"path": path, "file_gb": round(res.bam_len / 1e9, 3), "records": n}))


def run(path, window_gb, depth, reps, arena_factor, ramp=False):
    import torch  # noqa: F401 -- one HIP runtime
    from disq_amd import _lib, parallel as P, stream
    flen = os.path.getsize(path)
    with _lib.Context() as hc:
        header = hc.header_from_prefix(open(path, "rb").read(1 << 20))
    window = int(window_gb * 1e9)
    ctxs = []
    for _ in range(depth):
        c = _lib.Context()
        c.set_export_arena(int(window * arena_factor))
        ctxs.append(c)
    lk = threading.Lock()
    for rep in range(reps):
        got = {"records": 0, "raw": 0, "digests": []}

        def export(k, c, shard):
            b = c.read(with_raw=True)
            with lk:
                got["records"] += len(b["voffset"])
                got["raw"] += 0 if b["raw"] is None else len(b["raw"])
                got["digests"].append((shard.p0, b["part_digest"].copy()))
        res = stream.stream_read(path, flen, header, window=window, depth=depth,
                                 on_window=export, contexts=ctxs, ramp=ramp)
        dg = [0] * len(res["digests"])
        for p0, d in got["digests"]:
            for i, x in enumerate(d):
                dg[p0 + i] = int(x)
        secs = res["seconds"]
        print(json.dumps({
            "rep": rep, "mmap": os.environ.get("DQ_MMAP", "0"), "window_gb": window_gb,
            "depth": depth, "ramp": ramp, "windows": res["windows"], "seconds": round(secs, 3),
            "decompressed_gbs": round(res["owned_bytes"] / secs / 1e9, 2),
            "file_gbs": round(flen / secs / 1e9, 2),
            "open_h2d_s": round(res["open_s"], 3), "pipeline_s": round(res["run_s"], 3),
            "d2h_s": round(res["on_window_s"], 3), "records": got["records"],
            "digest": f"{res['digest']:016x}",
            "exported_digest_match": P.fold_digest(dg) == res["digest"]}), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("gen", "run"))
    ap.add_argument("path")
    ap.add_argument("gb", nargs="?", type=float, default=6.0)
    ap.add_argument("--window-gb", type=float, default=2.0)
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--arena-factor", type=float, default=3.7)
    ap.add_argument("--ramp", action="store_true")
    a = ap.parse_args()
    if a.mode == "gen":
        gen(a.path, a.gb)
    else:
        run(a.path, a.window_gb, a.depth, a.reps, a.arena_factor, a.ramp)
