set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r1g
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1g/pytest_gpu.log 2>&1 && tail -3 gpurun_out/r1g/pytest_gpu.log &&
for st in 0 2; do DQ_STORE=$st timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex inflate_block --output-format csv -d gpurun_out/r1g/wr$st -o run -- python3 -u bench.py --steps 1 --warmup 0 --cpu-seconds 1 --gb 2 > gpurun_out/r1g/wr$st.log 2>&1 || exit 1; done &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r1g/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 > gpurun_out/r1g/bench.log 2>&1 && tail -1 gpurun_out/r1g/bench.log
