#!/bin/bash
# Inflate kernel iteration check: GPU tests, then the default bench workload's K2 timing.
set -eo pipefail
out=gpurun_out/${1:-r2t}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $out/tests.log 2>&1
tail -1 $out/tests.log
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --cpu-seconds 1 --e2e 0 --intervals 0 > $out/bench.log 2>&1
grep '"metric"' $out/bench.log | tail -1 > $out/bench.json
python3 -c "import json;d=json.load(open('$out/bench.json'));print(d['value'],d['ms_per_step'],d['roofline'])"
