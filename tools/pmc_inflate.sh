#!/bin/bash
# Dev tool: PMC counter passes over the inflate kernel (one rocprofv3 run per pass).
# usage: tools/pmc_inflate.sh OUTDIR [NRECORDS]
set -e
out=${1:-gpurun_out/pmc}; n=${2:-2000000}
export TMPDIR=/tmp
mkdir -p "$out"
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
            "SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_UNALIGNED_STALL SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM" \
            "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "inflate_(block|tail)" --output-format csv -d $out/p$i -o run -- python3 -u tools/inflate_timing.py $n 3 > $out/p$i.log 2>&1
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(float); nd = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if 'inflate' not in r['Kernel_Name']: continue
        k = ('tail ' if 'inflate_tail' in r['Kernel_Name'] else 'block ') + r['Counter_Name']
        agg[k] += float(r['Counter_Value']); nd[k] += 1
for k in sorted(agg): print(f"{k:32s} {agg[k]:.4g}  (dispatch-rows {nd[k]})")
PY
