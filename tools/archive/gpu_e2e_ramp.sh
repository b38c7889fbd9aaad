#!/bin/bash
# End-to-end A/B: window ramp (small first and last windows) vs equal windows, 12.5 GB file in
# /dev/shm, interleaved.  usage: tools/gpu_e2e_ramp.sh TAG
set -eo pipefail
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/e2e_ab.py gen /dev/shm/e2e.bam 12.5 > $out/gen.log 2>&1
trap 'rm -f /dev/shm/e2e.bam' EXIT
timeout -k 10 300 python3 -u -m pytest tests/test_stream.py -m gpu -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for m in "" "--ramp"; do
    timeout -k 10 200 python3 -u tools/e2e_ab.py run /dev/shm/e2e.bam --window-gb 2 --depth 3 --reps 2 $m > $out/run${r}_${m:-eq}.log 2>&1
    echo "== ${m:-equal} rep $r"; grep "{" $out/run${r}_${m:-eq}.log | tail -2 | cut -c1-240
  done
done
