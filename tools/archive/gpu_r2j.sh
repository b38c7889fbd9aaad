#!/bin/bash
# Round-2 check of the spill-free inflate kernel: parity tests, phase cycles, a short bench, PMC passes.
set -eo pipefail
mkdir -p gpurun_out/r2j
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_chunk_decode.py > gpurun_out/r2j/tests.log 2>&1
DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 3 > gpurun_out/r2j/timing.log 2>&1
timeout -k 10 300 python3 -u bench.py --gb 2 --steps 3 --warmup 1 --cpu-seconds 1 --e2e 0 > gpurun_out/r2j/bench2.json 2> gpurun_out/r2j/bench2.log
bash tools/pmc_inflate.sh gpurun_out/r2j/pmc 2000000 > gpurun_out/r2j/pmc_summary.txt 2>&1
bash tools/pmc_traffic.sh gpurun_out/r2j/traffic gpurun_out/r2j/traffic.json --gb 2 --e2e 0 --intervals 0 > gpurun_out/r2j/traffic.log 2>&1
