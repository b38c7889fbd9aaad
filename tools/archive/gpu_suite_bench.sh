#!/bin/bash
# The whole -m gpu suite, then the default bench line.  usage: tools/gpu_suite_bench.sh TAG
set -eo pipefail
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -40 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
timeout -k 10 900 python3 -u bench.py > $out/bench_default.log 2>&1
grep '"metric"' $out/bench_default.log | tail -1 > $out/bench_default.json
python3 -c "
import json; d=json.load(open('$out/bench_default.json')); c=d['config']
print('value', d['value'], 'ms', d['ms_per_step'], 'k2', d['roofline']['avg_launch_ms'], c['device_ms_breakdown_rank0'], 'write', c['write_path']['input_gbs'], 'e2e', c['end_to_end']['seconds'], c['parity']['status'])"
