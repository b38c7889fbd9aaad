"""Dev tool: bench.py's end-to-end leg (page cache -> HBM -> pipeline -> host) over a list of
(window GB, depth, export) settings on one generated 12.5 GB configs[2]-shaped file, each run twice.

  python tools/e2e_sweep.py [--gb 12.5] 2:3:lean 2:4:lean 1:6:lean ... > out.jsonl
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=12.5)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("configs", nargs="+")
    a = ap.parse_args()
    import ctypes

    import numpy as np
    import torch  # noqa: F401
    import bench
    from disq_amd import _lib, synth
    probe = synth.generate(20000, seed=1, nthreads=16)
    n_total = int(a.gb * 1e9 / (len(probe.bam) / probe.n_records))
    t0 = time.time()
    res, free = synth.generate(n_total, seed=1, nthreads=16, as_buffer=True, unplaced_fraction=0.005)
    data = np.ctypeslib.as_array((ctypes.c_uint8 * res.bam_len).from_address(res.bam)).copy()
    free()
    print(f"generated {len(data) / 1e9:.2f} GB in {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    with _lib.Context() as hc:
        header = hc.header_from_prefix(bytes(data[:1 << 20]))
    for rep in range(a.reps):
        for cfg in a.configs:
            w, d, e = cfg.split(":")
            args = argparse.Namespace(e2e_window_gb=float(w), e2e_depth=int(d), e2e_export=e,
                                      split_size=0, no_crc=False)
            out = bench.end_to_end(data, args, None, header)
            out.pop("path", None)
            pc = out.pop("pcie_ceiling", {})
            print(json.dumps({"cfg": cfg, "rep": rep, "seconds": out.get("seconds"),
                              "gbs": out.get("decompressed_gbs"),
                              "stages": out.get("stage_seconds_summed_over_windows"),
                              "digest_ok": out.get("exported_digest_match"),
                              "frac_link": pc.get("frac_of_link_bound"),
                              "error": out.get("error")}), flush=True)


if __name__ == "__main__":
    main()
