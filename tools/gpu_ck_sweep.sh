#!/bin/bash
# Checkpoint spacing/count sweep: DQ_CKI/DQ_NCK pairs, plain + phase timing.  usage: TAG "cki:nck" ...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for cfg in "$@"; do
  c=${cfg%%:*}; n=${cfg##*:}
  DQ_CKI=$c DQ_NCK=$n timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain_$c.$n.log 2>&1
  DQ_CKI=$c DQ_NCK=$n DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing_$c.$n.log 2>&1
done
for f in $out/*.log; do echo "== $f"; grep -v "^bytes\|amdgpu.ids" $f | grep -o "inflate ms [0-9.]*\|spec=[0-9]*\|rounds=[0-9]*\|emit=[0-9]*" | tr '\n' ' '; echo; done
