#!/bin/bash
# Round-end validation in one call: smoke, the whole -m gpu suite, the bounds-checked run, the
# long-read checked run, then the default bench line.  usage: tools/gpu_final.sh TAG
set -eo pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
tools/gpu_full_then_checked.sh $tag
timeout -k 10 900 python3 -u bench.py > $out/bench_default.log 2>&1
grep '"metric"' $out/bench_default.log | tail -1 > $out/bench_default.json
python3 -c "
import json; d=json.load(open('$out/bench_default.json')); c=d['config']
print('value', d['value'], 'ms', d['ms_per_step'], 'k2', d['roofline']['avg_launch_ms'], c['device_ms_breakdown_rank0'], 'write', c['write_path']['input_gbs'], c['write_path']['ratio'], 'e2e', c['end_to_end']['seconds'], c['parity']['status'])"
