#!/bin/bash
set -eo pipefail
mkdir -p gpurun_out/r3s
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_adversarial.py tests/test_guesser_gpu.py tests/test_span.py tests/test_chunk_decode.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3s/tests.log 2>&1 || { tail -30 gpurun_out/r3s/tests.log; exit 1; }
tail -1 gpurun_out/r3s/tests.log
tools/gpu_deflate_ab.sh r3s_deflate
tools/gpu_prof_longread.sh r3s_lr 2
tools/gpu_e2e_ab.sh r3s_e2e 6
timeout -k 10 400 python3 -u bench.py --emulate-world 8 > gpurun_out/r3s/gen_n8.log 2>&1
tail -1 gpurun_out/r3s/gen_n8.log
