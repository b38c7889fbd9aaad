"""Dev tool: time the inflate kernel on a synthetic BAM (DQ_TIMING=1 prints per-phase cycles)."""
import sys, os, time
sys.path.insert(0, '/root/repo')
from disq_amd import _lib, synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000000
r = synth.generate(n, seed=1, nthreads=16)
print("bytes", len(r.bam), flush=True)
for ver in sys.argv[2:] or ["3"]:
    os.environ["DQ_INFLATE"] = ver
    with _lib.Context(split_size=0, verify_crc=True) as c:
        c.open_bytes(r.bam)
        st = c.run_resident()
        st = c.run_resident()
        print(ver, "inflate ms", st.ms_inflate, "total", st.ms_total, "records", st.ms_records,
              "ulen", st.decompressed_bytes, flush=True)
