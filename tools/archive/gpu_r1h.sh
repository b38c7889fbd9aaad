set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r1h
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1h/pytest_gpu.log 2>&1 && tail -3 gpurun_out/r1h/pytest_gpu.log &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r1h/smoke.log 2>&1 && tail -1 gpurun_out/r1h/smoke.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1h/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 > gpurun_out/r1h/bench.log 2>&1 && tail -1 gpurun_out/r1h/bench.log
