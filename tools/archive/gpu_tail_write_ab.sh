#!/bin/bash
# WRITE_SIZE and FETCH_SIZE of the inflate kernels (one rocprofv3 pass each) per library, on the
# 2M-record file.  usage: tools/gpu_tail_write_ab.sh TAG LIB...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for v in "$@"; do
  for c in WRITE_SIZE FETCH_SIZE; do
    DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "inflate_(block|tail)" \
      --output-format csv -d $out/pmc_${c}_$v -o run -- python3 -u tools/inflate_timing.py 2000000 1 > $out/pmc_${c}_$v.log 2>&1
  done
  python3 - $out $v <<'PY'
import csv, glob, sys, collections
out, v = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(float)
for c in ("WRITE_SIZE", "FETCH_SIZE"):
    for f in glob.glob(f"{out}/pmc_{c}_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = "tail" if "inflate_tail" in r["Kernel_Name"] else "block"
            agg[(k, c)] += float(r["Counter_Value"])
print(v, {f"{k}_{c}_KiB": round(x) for (k, c), x in sorted(agg.items())})
PY
done
