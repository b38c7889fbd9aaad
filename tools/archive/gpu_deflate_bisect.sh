#!/bin/bash
# Deflate GPU tests under several DQ_DEFLATE settings.  usage: CFGS="..." tools/gpu_deflate_bisect.sh TAG
out=gpurun_out/${1:-deflate_bisect}
mkdir -p $out
export TMPDIR=/tmp
for cfg in $CFGS; do
  DQ_DEFLATE=$cfg timeout -k 10 120 python3 -u -m pytest tests/test_deflate_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread > $out/t_$cfg.log 2>&1
  echo "$cfg: rc=$? $(tail -1 $out/t_$cfg.log)"
done
exit 0
