"""Dev tool: the records stage (record chain + SoA decode + hash) of the resident pipeline on a
synthetic WGS BAM of N records, K runs after one warm-up.  usage: tools/records_timing.py [N] [K]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from disq_amd import _lib, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
r = synth.generate(n, seed=1, nthreads=16)
print("bytes", len(r.bam), flush=True)
with _lib.Context(split_size=0, verify_crc=True) as c:
    c.open_bytes(r.bam)
    c.run_resident()
    ms = []
    for _ in range(k):
        st = c.run_resident()
        ms.append(st.ms_records)
        print("inflate ms %.3f records ms %.3f total %.3f ulen %d" % (st.ms_inflate, st.ms_records, st.ms_total,
                                                                     st.decompressed_bytes), flush=True)
    print("records ms median %.3f" % sorted(ms)[len(ms) // 2])
checked, fails = _lib.checked_report()
if checked:
    print("checked build:", fails or "no failed device checks")
