#!/bin/bash
# Dev tool: PMC counter passes over the deflate kernels (bgzf_parse/huff/code_kernel), one
# rocprofv3 run per pass, over tools/deflate_bench.py.  usage: tools/pmc_deflate.sh OUTDIR [NRECORDS]
set -e
out=${1:-gpurun_out/pmc_deflate}; n=${2:-500000}
export TMPDIR=/tmp
mkdir -p "$out"
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
            "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_WR SQ_LDS_UNALIGNED_STALL SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_WR" \
            "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "bgzf_(parse|huff|code)" --output-format csv -d $out/p$i -o run -- python3 -u tools/deflate_bench.py --records $n --reps 1 > $out/p$i.log 2>&1
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(float); nd = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        kn = r['Kernel_Name']
        k = ("parse" if "parse" in kn else "huff" if "huff" in kn else "code", r['Counter_Name'])
        agg[k] += float(r['Counter_Value']); nd[k] += 1
for k in sorted(agg): print(f"{k[0]:6s} {k[1]:28s} {agg[k]:.4g}  (dispatch-rows {nd[k]})")
# HBM traffic per input byte (MI355X_MICROARCH.md: FETCH_SIZE x 2 on gfx950; both in KiB)
import json, re
gb = zgb = None
for line in open(out + "/p1.log"):
    if line.startswith("{") and '"input_gb"' in line:
        j = json.loads(line)
        gb, zgb = j["input_gb"], j["compressed_gb"]
if gb:
    tot = 0.0
    for kn in ("parse", "huff", "code"):
        # (deflate_bench.py --reps 1 compresses the stream twice: a warm-up and the timed rep)
        f, w = agg.get((kn, "FETCH_SIZE"), 0.0) * 1024, agg.get((kn, "WRITE_SIZE"), 0.0) * 1024 / 2
        tot += f + w
        print(f"traffic {kn:6s} fetch {f / 1e9:.3f} GB  write {w / 1e9:.3f} GB  ({(f + w) / (gb * 1e9):.2f}x input)")
    print(f"traffic total {tot / 1e9:.3f} GB over {gb} GB of input (one rep): {tot / (gb * 1e9):.2f}x")
    print(f"algorithmic bytes (input read + output written) {gb + zgb:.3f} GB: traffic {tot / ((gb + zgb) * 1e9):.2f}x")
PY
