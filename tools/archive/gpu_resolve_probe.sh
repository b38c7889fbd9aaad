#!/bin/bash
# Resolve development probe: DQ_TIMING phase table of the current library (default and DQ_RPRIO=1),
# plain inflate timings interleaved with a reference library, and PMC instruction counts of both.
# usage: tools/gpu_resolve_probe.sh TAG REFLIB
set -eo pipefail
tag=$1; ref=$2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in libdisq_gpu.so $ref; do
    DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain${rep}_$v.log 2>&1
  done
  DQ_RPRIO=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain${rep}_prio.log 2>&1
done
DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing.log 2>&1
DQ_TIMING=1 DQ_RPRIO=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing_prio.log 2>&1
for v in libdisq_gpu.so $ref; do
  DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    --kernel-include-regex "inflate_block" --output-format csv -d $out/pmc_$v -o run -- \
    python3 -u tools/inflate_timing.py 2000000 > $out/pmc_$v.log 2>&1
done
for f in $out/*.log; do echo "== $f"; grep -v "^bytes\|amdgpu.ids\|^\[rocprof" $f | tail -5 || true; done
python3 - $out <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for d in sorted(glob.glob(out + "/pmc_*/")):
    agg = collections.defaultdict(float)
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r['Counter_Name']] += float(r['Counter_Value'])
    print(d, {k: f"{v:.4g}" for k, v in sorted(agg.items())})
PY
