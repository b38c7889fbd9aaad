#!/bin/bash
# GPU tests (a pytest -k selection, or all when empty) into gpurun_out/TAG/tests.log, then an
# optional command.  usage: tools/gpu_tests_then.sh TAG "pytest -k expr" [command...]
set -eo pipefail
tag=$1; sel=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ -n "$sel" ]; then k=(-k "$sel"); else k=(); fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
if [ $# -gt 0 ]; then "$@"; fi
