#!/bin/bash
# tools/gpu_check.sh plus a rocprofv3 kernel trace of a short bench run (per-kernel breakdown).
set -eo pipefail
tag=${1:-checkprof}
bash tools/gpu_check.sh $tag
out=gpurun_out/$tag
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 1 --e2e 0 --intervals 0 > $out/prof_bench.log 2>&1
find $out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/kernel_stats.csv
head -14 $out/kernel_stats.csv | cut -c1-160
