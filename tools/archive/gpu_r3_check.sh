#!/bin/bash
# Round-3 check: GPU suite, the default bench (end-to-end included), the long-read bench (configs[4]).
# usage: tools/gpu_r3_check.sh TAG [LONGREAD_GB]
set -eo pipefail
tag=${1:-r3}; lgb=${2:-2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
tail -2 $out/gpu_tests.log
timeout -k 10 600 python3 -u bench.py > $out/bench.log 2>&1
grep '"metric"' $out/bench.log > $out/bench.json
python3 -c "import json;d=json.load(open('$out/bench.json'));c=d['config'];print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],c['parity']['status'],json.dumps(c['interval_mode'].get('parity',{}).get('status')),json.dumps(c['end_to_end']))"
if [ "$lgb" != 0 ]; then
  timeout -k 10 400 python3 -u bench.py --shape longread --gb $lgb --cpu-seconds 8 --e2e 0 > $out/bench_longread.log 2>&1
  grep '"metric"' $out/bench_longread.log > $out/bench_longread.json
  python3 -c "import json;d=json.load(open('$out/bench_longread.json'));c=d['config'];print(d['value'],d['ms_per_step'],c['reads_per_s'],c['parity']['status'],json.dumps(c['device_ms_breakdown_rank0']))"
fi
