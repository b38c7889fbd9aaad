#!/bin/bash
set -eo pipefail
mkdir -p gpurun_out/r3t
export TMPDIR=/tmp
tools/gpu_deflate_ab.sh r3t_deflate
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3t/dprof -o run -- python3 -u tools/deflate_bench.py > gpurun_out/r3t/deflate_prof.log 2>&1
find gpurun_out/r3t/dprof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r3t/deflate_kernel_stats.csv
head -4 gpurun_out/r3t/deflate_kernel_stats.csv | cut -c1-200
timeout -k 10 600 python3 -u bench.py > gpurun_out/r3t/bench.log 2>&1
grep '"metric"' gpurun_out/r3t/bench.log > gpurun_out/r3t/bench.json
python3 -c "import json;d=json.load(open('gpurun_out/r3t/bench.json'));c=d['config'];print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],c['parity']['status'],c['device_ms_breakdown_rank0'],json.dumps(c['end_to_end']))"
