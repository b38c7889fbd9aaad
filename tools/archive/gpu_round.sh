#!/bin/bash
# One GPU round trip: inflate timing (plain x2 + DQ_TIMING phase cycles) on the 2M-record file, the
# GPU suite, and a short 12.5 GB bench with interval mode + oracle parity.  usage: tools/gpu_round.sh TAG
set -eo pipefail
tag=${1:-round}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain.log 2>&1
DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing.log 2>&1
timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain2.log 2>&1
grep -hv "^bytes\|amdgpu.ids" $out/plain.log $out/timing.log $out/plain2.log
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
tail -2 $out/gpu_tests.log
if [ "${BENCH:-1}" != 0 ]; then
  timeout -k 10 500 python3 -u bench.py --steps 5 --warmup 2 --cpu-seconds 8 --e2e 0 > $out/bench.log 2>&1
  grep '"metric"' $out/bench.log > $out/bench.json
  grep "step 4" $out/bench.log
  python3 -c "import json;d=json.load(open('$out/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['config']['parity']['status'],json.dumps(d['config']['interval_mode'].get('parity')))"
fi
