#!/bin/bash
# Deflate tests on the default library and, with chains up to 128 (libdisq_gpu_mc128.so), at long
# chains with lazy matching; then ratio / speed at those settings.  usage: tools/gpu_deflate_fixcheck.sh TAG
out=gpurun_out/${1:-deflate_fix}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python3 -u -m pytest tests/test_deflate_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread > $out/t_default.log 2>&1
echo "default: rc=$? $(tail -1 $out/t_default.log)"
for cfg in 96,32,96,8 80,24,48,8 128,32,128,16 96,32,96,0; do
  DQ_GPU_LIB=$PWD/disq_amd/_build/libdisq_gpu_mc128.so DQ_DEFLATE=$cfg timeout -k 10 120 python3 -u -m pytest tests/test_deflate_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread > $out/t_$cfg.log 2>&1
  echo "$cfg: rc=$? $(tail -1 $out/t_$cfg.log)"
done
for cfg in 96,32,96,8 80,32,80,8; do
  DQ_GPU_LIB=$PWD/disq_amd/_build/libdisq_gpu_mc128.so DQ_DEFLATE=$cfg timeout -k 10 200 python3 -u tools/deflate_bench.py > $out/bench_$cfg.log 2>&1
  echo "$cfg: $(grep '"ratio"' $out/bench_$cfg.log)"
done
exit 0
