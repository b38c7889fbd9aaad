"""GPU BGZF compression throughput (write path): the resident
decompressed stream of a synthetic WGS-shaped BAM compressed into 65280-byte BGZF blocks.

  python tools/deflate_bench.py [--records 2000000] [--reps 3] > out.json

Reports input GB/s over the device time (HIP events around the deflate + pack kernels),
the compression ratio, and a round trip: the output re-inflated by the GPU inflate kernel (read
as a BGZF text stream) must reproduce the input bytes (digest of both streams)."""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=2000000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch  # noqa: F401 -- one HIP runtime
    from disq_amd import _lib, synth
    r = synth.generate(a.records, seed=1, nthreads=16)
    eof = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    with _lib.Context(verify_crc=True) as c:
        c.open_bytes(r.bam)
        c.run_resident()
        u = c.inflated()
        runs = [c.bgzf_compress_resident() for _ in range(a.reps + 1)]
        n = runs[-1][0]
        z = c.bgzf_fetch(n).tobytes()
    ms = sorted(x[1] for x in runs[1:])[len(runs[1:]) // 2]
    with _lib.Context(verify_crc=True) as c:
        c.text_open_bytes(z + eof)
        c.text_run(False)
        back = c.inflated()
    ok = hashlib.sha256(u.tobytes()).hexdigest() == hashlib.sha256(back.tobytes()).hexdigest()
    out = {"input_gb": round(len(u) / 1e9, 4), "compressed_gb": round(n / 1e9, 4),
           "ratio": round(len(u) / n, 3), "device_ms_median": round(ms, 3),
           "input_gbs": round(len(u) / ms / 1e6, 2), "reps": a.reps,
           "htsjdk_level5_ratio": round(len(u) / len(r.bam), 3),
           "roundtrip_gpu_inflate": "match" if ok else "MISMATCH"}
    print(json.dumps(out), flush=True)
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
