#!/bin/bash
# Guesser round (r6y): record-path GPU tests and the checked build on the product, records timing
# of the product against the previous check_internal (ck0), a long-read bench run for its parity.
o=gpurun_out/${1:-r6y}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_adversarial.py tests/test_guesser_gpu.py tests/test_lean_export.py tests/test_parallel.py tests/test_chunk_decode.py -m gpu -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
DQ_GPU_LIB=$PWD/disq_amd/_build/libdisq_gpu_checked.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_adversarial.py tests/test_guesser_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $o/checked_tests.log 2>&1 || { tail -30 $o/checked_tests.log; exit 1; }
tail -1 $o/checked_tests.log
for rep in 1 2; do for v in libdisq_gpu_ck0.so libdisq_gpu.so; do DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -k 10 200 python3 -u tools/records_timing.py 20000000 5 > $o/rt${rep}_$v.log 2>&1 || exit 1; echo "$rep $v $(tail -1 $o/rt${rep}_$v.log)"; done; done
timeout -k 10 600 python3 -u bench.py --shape longread --gb 2 --steps 3 --warmup 1 --e2e 0 --intervals 0 --cpu-seconds 1 > $o/longread.log 2>&1 || { tail -20 $o/longread.log; exit 1; }
grep '"metric"' $o/longread.log | tail -1 > $o/longread.json
python3 -c "import json; d=json.load(open('$o/longread.json')); print('longread', d['value'], d['config']['device_ms_breakdown_rank0'], d['config']['parity']['status'])"
