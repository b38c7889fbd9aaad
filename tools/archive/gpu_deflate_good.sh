#!/bin/bash
# Deflate (row f3): GPU tests, then ratio / throughput with the lazy look-ahead's chain cut at
# `good` (DQ_DEFLATE="chain,lazy,nice,good"; good 0 = the full chain).  usage: tools/gpu_deflate_good.sh TAG
set -eo pipefail
out=gpurun_out/${1:-deflate_good}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_deflate_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for cfg in ${CFGS:-"48,24,48,0" "48,24,48,8" "48,24,48,16" "64,32,64,8" "48,32,64,8"}; do
  DQ_DEFLATE=$cfg timeout -k 10 200 python3 -u tools/deflate_bench.py > $out/bench_$cfg.log 2>&1
  echo "$cfg: $(grep '"ratio"' $out/bench_$cfg.log)"
done
