#!/bin/bash
# HBM traffic of the inflate kernel (bench.py's dominant kernel): two rocprofv3 PMC passes over a
# short bench run, FETCH_SIZE and WRITE_SIZE separately (they do not fit one pass), summarised per
# launch into $2 (JSON).  gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts 64 B per
# 128-B request, so it is doubled; both counters are in KiB.
# usage: tools/pmc_traffic.sh OUTDIR SUMMARY.json [bench args...]
set -e
out=${1:-gpurun_out/pmc_traffic}; summary=${2:-$out/summary.json}; shift 2 || true
export TMPDIR=/tmp
mkdir -p "$out"
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex inflate_block --output-format csv \
  -d "$out/fetch" -o run -- python3 -u bench.py --steps 1 --warmup 0 --cpu-seconds 1 "$@" > "$out/fetch.log" 2>&1
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex inflate_block --output-format csv \
  -d "$out/write" -o run -- python3 -u bench.py --steps 1 --warmup 0 --cpu-seconds 1 "$@" > "$out/write.log" 2>&1
python3 - "$out" "$summary" <<'PY'
import csv, glob, json, sys
out, summary = sys.argv[1], sys.argv[2]
vals = {}
for name in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = []
    for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "inflate_block" in r["Kernel_Name"] and r["Counter_Name"] == name:
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    per = {}
    for d, v in rows:
        per[d] = per.get(d, 0.0) + v
    vals[name] = sorted(per.values())
fetch = [2 * 1024 * v for v in vals["FETCH_SIZE"]]
write = [1024 * v for v in vals["WRITE_SIZE"]]
res = {"kernel": "inflate_block_kernel", "launches": len(fetch),
       "fetch_bytes_per_launch": max(fetch) if fetch else None,
       "write_bytes_per_launch": max(write) if write else None,
       "correction": "FETCH_SIZE x2 (gfx950: 64 B tallied per 128-B request), KiB -> bytes",
       "raw_FETCH_SIZE_KiB": vals["FETCH_SIZE"], "raw_WRITE_SIZE_KiB": vals["WRITE_SIZE"]}
if fetch and write:
    res["traffic_bytes_per_launch"] = max(fetch) + max(write)
json.dump(res, open(summary, "w"), indent=1)
print(json.dumps(res))
PY
