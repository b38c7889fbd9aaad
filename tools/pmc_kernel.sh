#!/bin/bash
# PMC passes (one rocprofv3 run each) over the kernels matching a regex, on the 2M-record file
# (tools/records_timing.py runs the whole pipeline).  usage: tools/pmc_kernel.sh OUTDIR REGEX [NRECORDS]
set -e
out=$1; rx=$2; n=${3:-2000000}
export TMPDIR=/tmp
mkdir -p "$out"
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
            "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "$rx" --output-format csv -d $out/p$i -o run -- python3 -u tools/records_timing.py $n 1 > $out/p$i.log 2>&1
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(float); nd = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0][-40:] + ' ' + r['Counter_Name']
        agg[k] += float(r['Counter_Value']); nd[k] += 1
for k in sorted(agg): print(f"{k:70s} {agg[k]:.4g}  (rows {nd[k]})")
PY
