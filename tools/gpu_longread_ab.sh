#!/bin/bash
# Long-read (configs[4]) A/B of prebuilt libraries: bench.py --shape longread, interleaved twice.
# usage: tools/gpu_longread_ab.sh TAG LIB...
set -eo pipefail
tag=$1; shift; o=gpurun_out/$tag; mkdir -p $o; export TMPDIR=/tmp
for rep in 1 2; do for v in "$@"; do
  DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -k 10 400 python3 -u bench.py --shape longread --gb 2 --steps 5 --warmup 2 --e2e 0 --intervals 0 --cpu-seconds 0 > $o/lr${rep}_$v.log 2>&1 || { tail -20 $o/lr${rep}_$v.log; exit 1; }
  grep '"metric"' $o/lr${rep}_$v.log | tail -1 > $o/lr${rep}_$v.json
  python3 -c "import json; d=json.load(open('$o/lr${rep}_$v.json')); print('$rep $v', d['value'], d['config']['device_ms_breakdown_rank0'], (d['config'].get('parity') or {}).get('status'))"
done; done
