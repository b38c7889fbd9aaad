#!/bin/bash
# One GPU call for a kernel-variant round: the inflate parity tests under each variant library,
# the interleaved A/B of the product library against them (tools/gpu_variant_ab.sh), then the
# whole -m gpu suite and the default bench line on the product library.  Stops at the first
# failure.  usage: tools/gpu_ab_then_suite.sh TAG [VARIANT_LIB...]   (names under disq_amd/_build)
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for v in "$@"; do
  DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
    tests/test_inflate_codes.py tests/test_tail_handoff.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > $out/tests_$v.log 2>&1 || { tail -30 $out/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $out/tests_$v.log)"
done
if [ $# -gt 0 ]; then tools/gpu_variant_ab.sh $tag libdisq_gpu.so "$@"; fi
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -40 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
timeout -k 10 600 python3 -u bench.py > $out/bench_default.log 2>&1
grep '"metric"' $out/bench_default.log | tail -1 > $out/bench_default.json
python3 -c "
import json; d=json.load(open('$out/bench_default.json')); c=d['config']
print('value', d['value'], 'ms', d['ms_per_step'], 'k2', d['roofline']['avg_launch_ms'], c['device_ms_breakdown_rank0'], 'write', c['write_path']['input_gbs'], 'e2e', c['end_to_end'].get('seconds'), c['end_to_end'].get('decompressed_gbs'), c['parity']['status'])"
