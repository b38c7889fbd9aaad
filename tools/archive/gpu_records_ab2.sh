#!/bin/bash
# Records-stage variants (r6n): the speculation's phase timing (-DDQ_REC_TIMING), then interleaved
# records timing of the product library against non-temporal SoA stores and 4 lanes per record.
o=gpurun_out/${1:-r6n}; mkdir -p $o; export TMPDIR=/tmp
DQ_GPU_LIB=$PWD/disq_amd/_build/libdisq_gpu_rth.so timeout -k 10 200 python3 -u tools/records_timing.py 20000000 2 > $o/tim_rth.log 2>&1 || exit 1
grep "seg_spec cycles\|decode_records cycles" $o/tim_rth.log | tail -2
for rep in 1 2; do for v in libdisq_gpu.so libdisq_gpu_rnt.so libdisq_gpu_rl4.so; do DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -k 10 200 python3 -u tools/records_timing.py 20000000 5 > $o/rt${rep}_$v.log 2>&1 || exit 1; echo "$rep $v $(tail -1 $o/rt${rep}_$v.log)"; done; done
