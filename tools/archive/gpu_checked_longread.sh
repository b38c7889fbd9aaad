set -eo pipefail
mkdir -p gpurun_out/r4e
export TMPDIR=/tmp DQ_GPU_LIB=$PWD/disq_amd/_build/libdisq_gpu_checked.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_chunk_decode.py -m gpu -v -s --timeout 200 --timeout-method thread -k "long" > gpurun_out/r4e/chk.log 2>&1 || true
grep "DQ_CHECKED\]\|passed\|failed" gpurun_out/r4e/chk.log | tail -5
