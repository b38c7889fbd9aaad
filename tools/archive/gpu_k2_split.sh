#!/bin/bash
# rocprofv3 kernel trace of the inflate kernels (block + tail) for each given library, on the
# WGS file of DQ_N records (default 2M): per-kernel average durations.
# usage: [DQ_N=...] tools/gpu_k2_split.sh TAG LIB...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/kt${i}_$v -o run -- \
    python3 -u tools/inflate_timing.py ${DQ_N:-2000000} > $out/kt${i}_$v.log 2>&1
done
i=0
for v in "$@"; do
  i=$((i+1))
  echo "== $v"
  f=$(find $out/kt${i}_$v -name "*kernel_stats.csv" | head -1)
  if [ -z "$f" ]; then  # (this rocprofv3 writes a rocpd database by default)
    db=$(find $out/kt${i}_$v -name "*.db" | head -1)
    f=$out/kt${i}_$v/kernel_stats.csv
    python3 tools/rocpd_stats.py "$db" "$f" > /dev/null
  fi
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'inflate' in r['Name'] or 'decode_records' in r['Name']:
        print(f"{r['Name'][:60]:60s} calls {r['Calls']:>4s} avg_ms {float(r['AverageNs'])/1e6:.3f}")
PY
done
