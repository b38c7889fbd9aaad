#!/bin/bash
# Records-stage round (r6o): the checked build (speculation equivalence), record-path GPU tests,
# the speculation's phase timing, interleaved records timing (sw0: full checks on U; product: from
# the LDS window; rnt: + non-temporal SoA stores), kernel trace of the product.
o=gpurun_out/${1:-r6o}; mkdir -p $o; export TMPDIR=/tmp
DQ_GPU_LIB=$PWD/disq_amd/_build/libdisq_gpu_checked.so timeout -k 10 200 python3 -u tools/records_timing.py 2000000 1 > $o/checked_rt.log 2>&1 || { tail $o/checked_rt.log; exit 1; }
tail -1 $o/checked_rt.log
DQ_GPU_LIB=$PWD/disq_amd/_build/libdisq_gpu_checked.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_adversarial.py tests/test_guesser_gpu.py tests/test_lean_export.py -m gpu -q --timeout 300 --timeout-method thread > $o/checked_tests.log 2>&1 || { tail -30 $o/checked_tests.log; exit 1; }
tail -1 $o/checked_tests.log
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_adversarial.py tests/test_guesser_gpu.py tests/test_lean_export.py tests/test_parallel.py tests/test_chunk_decode.py -m gpu -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
DQ_GPU_LIB=$PWD/disq_amd/_build/libdisq_gpu_rth.so timeout -k 10 200 python3 -u tools/records_timing.py 20000000 2 > $o/tim_rth.log 2>&1 || exit 1
grep "seg_spec cycles" $o/tim_rth.log | tail -1
for rep in 1 2; do for v in libdisq_gpu_sp0.so libdisq_gpu_sw0.so libdisq_gpu.so libdisq_gpu_rnt.so; do DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -k 10 200 python3 -u tools/records_timing.py 20000000 5 > $o/rt${rep}_$v.log 2>&1 || exit 1; echo "$rep $v $(tail -1 $o/rt${rep}_$v.log)"; done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 -u tools/records_timing.py 20000000 3 > $o/prof.log 2>&1
