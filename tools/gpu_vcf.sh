#!/bin/bash
# Row f4 (BGZF text / VCF): GPU text tests, then tools/vcf_bench.py on a sites-only and a
# 200-sample synthetic VCF, the second under a rocprofv3 kernel trace.  usage: tools/gpu_vcf.sh TAG
set -eo pipefail
out=gpurun_out/${1:-vcf}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_text_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 400 python3 -u tools/vcf_bench.py --mb 4096 --samples 0 > $out/sites.log 2>&1
grep '"metric"' $out/sites.log > $out/sites.json; cut -c1-400 $out/sites.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 -u tools/vcf_bench.py --mb 4096 --samples 200 > $out/gt.log 2>&1
grep '"metric"' $out/gt.log > $out/gt.json; cut -c1-400 $out/gt.json
find $out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/kernel_stats.csv
head -8 $out/kernel_stats.csv | cut -c1-150
