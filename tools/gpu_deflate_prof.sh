#!/bin/bash
# Write path (row f3) evidence: rocprofv3 kernel trace + stats of tools/deflate_bench.py, and the
# deflate kernel's HBM traffic (FETCH_SIZE and WRITE_SIZE passes).  usage: tools/gpu_deflate_prof.sh TAG
set -eo pipefail
out=gpurun_out/${1:-deflate_prof}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_deflate_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
tail -1 $out/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 -u tools/deflate_bench.py --records 2000000 --reps 3 > $out/bench.log 2>&1
grep '"ratio"' $out/bench.log > $out/bench.json
find $out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/kernel_stats.csv
head -6 $out/kernel_stats.csv | cut -c1-160
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "bgzf_(parse|code)" --output-format csv -d $out/$c -o run -- \
    python3 -u tools/deflate_bench.py --records 2000000 --reps 1 > $out/$c.log 2>&1
done
python3 - $out <<'PY'
import csv, glob, sys
out = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            print(c, r["Kernel_Name"][:60], r["Counter_Value"])
PY
