#!/bin/bash
# The CPU oracle tests against the AddressSanitizer + UBSan build of oracle/disq_oracle.c (host code
# only, this container).  The interpreter is not instrumented, so the ASan runtime is preloaded;
# leak checks are off (CPython's own allocations would drown the report).
# usage: tools/oracle_asan.sh LOG
set -o pipefail
log=${1:-profiles/r3_oracle_asan.log}
make -s -C oracle asan
export DQ_ORACLE_LIB=$PWD/oracle/_build/libdisq_oracle_asan.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" \
  python3 -m pytest -q -m "not gpu" -p no:cacheprovider \
  tests/test_oracle_golden.py tests/test_splits_and_synth.py tests/test_sbi.py \
  tests/test_text_oracle.py tests/test_span_oracle.py tests/test_parallel.py > "$log" 2>&1
rc=$?
echo "exit $rc ($DQ_ORACLE_LIB)" >> "$log"
tail -3 "$log"
exit $rc
