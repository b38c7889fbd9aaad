#!/bin/bash
# Dev tool: inflate time and WRITE_SIZE per DQ_STORE mode on the 2M-record synthetic file.
export TMPDIR=/tmp
for m in 0 1 2 3; do
  DQ_STORE=$m timeout -k 10 100 python3 -u tools/inflate_timing.py 2000000 3 2>&1 | grep inflate
  DQ_STORE=$m timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex inflate_block --output-format csv -d gpurun_out/wpmc$m -o run -- python3 -u tools/inflate_timing.py 2000000 3 > /dev/null 2>&1
  python3 -c "
import csv,glob
v=[float(r['Counter_Value']) for f in glob.glob('gpurun_out/wpmc$m/**/*counter_collection.csv',recursive=True) for r in csv.DictReader(open(f)) if r['Counter_Name']=='WRITE_SIZE']
print('mode $m WRITE_SIZE KiB per launch', [round(x) for x in v])"
done
