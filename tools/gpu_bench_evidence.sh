#!/bin/bash
# Round evidence in one call: tools/gpu_evidence.sh (rocprof kernel trace of the bench workload,
# K2 HBM traffic, K2 SQ counters), then the default bench.py line (end-to-end leg, PCIe ceiling,
# write path).  usage: tools/gpu_bench_evidence.sh TAG
set -eo pipefail
tag=$1
out=gpurun_out/$tag
tools/gpu_evidence.sh $tag
timeout -k 10 900 python3 -u bench.py > $out/bench_default.log 2>&1
grep '"metric"' $out/bench_default.log | tail -1 > $out/bench_default.json
head -c 400 $out/bench_default.json; echo
