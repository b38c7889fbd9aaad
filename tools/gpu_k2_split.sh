#!/bin/bash
# rocprofv3 kernel trace of the inflate kernels (block + tail) for each given library, on the
# 2M-record WGS file: per-kernel average durations.  usage: tools/gpu_k2_split.sh TAG LIB...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for v in "$@"; do
  DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/kt_$v -o run -- \
    python3 -u tools/inflate_timing.py 2000000 > $out/kt_$v.log 2>&1
done
for v in "$@"; do
  echo "== $v"
  f=$(find $out/kt_$v -name "*kernel_stats.csv" | head -1)
  if [ -z "$f" ]; then  # (this rocprofv3 writes a rocpd database by default)
    db=$(find $out/kt_$v -name "*.db" | head -1)
    f=$out/kt_$v/kernel_stats.csv
    python3 tools/rocpd_stats.py "$db" "$f" > /dev/null
  fi
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'inflate' in r['Name'] or 'decode_records' in r['Name']:
        print(f"{r['Name'][:60]:60s} calls {r['Calls']:>4s} avg_ms {float(r['AverageNs'])/1e6:.3f}")
PY
done
