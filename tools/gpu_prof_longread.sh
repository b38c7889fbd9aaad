#!/bin/bash
# rocprofv3 kernel trace of the long-read bench (configs[4] shape): per-kernel breakdown.
# usage: tools/gpu_prof_longread.sh TAG [GB]
set -eo pipefail
tag=${1:-lrprof}; gb=${2:-2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 -u bench.py --shape longread --gb $gb --steps 2 --warmup 1 --cpu-seconds 1 --e2e 0 > $out/prof_bench.log 2>&1
find $out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/kernel_stats.csv
head -24 $out/kernel_stats.csv | cut -c1-200
