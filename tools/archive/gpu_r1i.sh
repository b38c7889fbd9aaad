set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r1i
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1i/pytest_gpu.log 2>&1 && tail -3 gpurun_out/r1i/pytest_gpu.log &&
timeout -k 10 200 python3 -u bench.py --gb 1 --steps 2 --warmup 1 --cpu-seconds 1 > gpurun_out/r1i/bench_small.log 2>&1 && tail -1 gpurun_out/r1i/bench_small.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1i/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 > gpurun_out/r1i/bench.log 2>&1 && grep '"metric"' gpurun_out/r1i/bench.log
