#!/bin/bash
# Round-3 extra evidence: rocprof of the deflate kernel (write path) and the 40 GB out-of-core read.
set -eo pipefail
out=gpurun_out/${1:-r3extra}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/dprof -o run -- python3 -u tools/deflate_bench.py > $out/deflate_prof.log 2>&1
find $out/dprof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/deflate_kernel_stats.csv
grep '"ratio"' $out/deflate_prof.log; grep -i "deflate\|pack" $out/deflate_kernel_stats.csv | cut -c1-160
timeout -k 10 700 python3 -u tools/stream_bench.py --gb 40 --window-gb 4 --depth 3 > $out/stream_40gb.log 2>&1
tail -1 $out/stream_40gb.log
