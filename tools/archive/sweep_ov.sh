set -o pipefail
mkdir -p gpurun_out/sweep2
run() { timeout -k 10 120 python3 -u bench.py --gb 2 --steps 3 --warmup 1 --cpu-seconds 0 --intervals 0 > gpurun_out/sweep2/$1.log 2>&1 || exit 1
  echo "$1 $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/sweep2/$1.log) $(grep -o '"digest_rank0": "[0-9a-f]*"' gpurun_out/sweep2/$1.log)"; }
for ov in 32 48 64 80; do DQ_OV=$ov run ov$ov; done
for cfg in 4,4 2,4 1,4; do DQ_OV=64 DQ_CFG=$cfg run cfg${cfg/,/_}; done
