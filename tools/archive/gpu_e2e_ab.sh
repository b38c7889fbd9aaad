#!/bin/bash
# End-to-end A/B: one file in /dev/shm, the upload path (registered mapping vs pinned staging) and
# window/depth settings, each in its own process.  usage: tools/gpu_e2e_ab.sh TAG [GB]
set -eo pipefail
tag=${1:-e2e}; gb=${2:-6}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
f=/dev/shm/dq_e2e_$$.bam
trap 'rm -f $f' EXIT
timeout -k 10 200 python3 -u tools/e2e_ab.py gen $f $gb > $out/gen.log 2>&1
tail -1 $out/gen.log
for cfg in "1 2 3" "0 2 3" "1 1 4" "0 1 4" "0 0.5 6"; do
  set -- $cfg
  DQ_MMAP=$1 timeout -k 10 120 python3 -u tools/e2e_ab.py run $f --window-gb $2 --depth $3 --reps 2 \
    > $out/run_$1_$2_$3.log 2>&1
  grep '"rep"' $out/run_$1_$2_$3.log
done
