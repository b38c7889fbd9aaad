#!/bin/bash
# Deflate (write path, row f3): GPU tests, then ratio / throughput at several match-search
# settings (DQ_DEFLATE="chain,lazy,nice").  usage: tools/gpu_deflate_ab.sh TAG
set -eo pipefail
tag=${1:-deflate}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_deflate_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for cfg in "48,24,48" "32,16,32" "64,32,64" "16,8,16"; do
  DQ_DEFLATE=$cfg DQ_DEFLATE_TIMING=1 timeout -k 10 200 python3 -u tools/deflate_bench.py > $out/bench_$cfg.log 2>&1
  echo "$cfg: $(grep '"ratio"' $out/bench_$cfg.log)"
  grep "deflate phase" $out/bench_$cfg.log | tail -1
done
