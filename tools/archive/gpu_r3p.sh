set -eo pipefail
mkdir -p gpurun_out/r3p
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_adversarial.py tests/test_guesser_gpu.py tests/test_parallel.py tests/test_span.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3p/tests.log 2>&1
tail -1 gpurun_out/r3p/tests.log
tools/gpu_prof_longread.sh r3p 2
tools/gpu_e2e_ab.sh r3p_e2e 6
DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > gpurun_out/r3p/timing.log 2>&1
grep "\[dq\]" gpurun_out/r3p/timing.log
timeout -k 10 400 python3 -u bench.py --emulate-world 8 > gpurun_out/r3p/gen_n8.log 2>&1
tail -1 gpurun_out/r3p/gen_n8.log
