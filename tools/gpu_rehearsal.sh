#!/bin/bash
# bench.py --gpus N rehearsal on a one-GPU box (DQ_BENCH_REHEARSAL=1: gloo collectives, every rank
# on GPU 0 -- RCCL refuses two ranks on one device): the N > 1 logic end to end, with the per-rank
# oracle parity.  Values are NOT measurements.  usage: tools/gpu_rehearsal.sh TAG GB N...
set -eo pipefail
tag=$1; gb=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp DQ_BENCH_REHEARSAL=1
for n in "$@"; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 \
    --gb $gb --intervals 0 --e2e 0 --cpu-seconds 0 > $out/rehearsal_n$n.json 2> $out/rehearsal_n$n.log
  echo "n=$n: $(python3 -c "import json,sys; d=json.loads(open('$out/rehearsal_n$n.json').read().strip().splitlines()[-1]); print(json.dumps(d['config']['parity']))")"
done
