#!/bin/bash
# HBM traffic of the inflate (K2: inflate_block_kernel + inflate_tail_kernel, bench.py's dominant
# kernels): two rocprofv3 PMC passes over a
# short bench run, FETCH_SIZE and WRITE_SIZE separately (they do not fit one pass), summarised per
# launch into $2 (JSON).  gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts 64 B per
# 128-B request, so it is doubled; both counters are in KiB.
# usage: tools/pmc_traffic.sh OUTDIR SUMMARY.json [bench args...]
set -e
out=${1:-gpurun_out/pmc_traffic}; summary=${2:-$out/summary.json}; shift 2 || true
export TMPDIR=/tmp
mkdir -p "$out"
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "inflate_(block|tail)" --output-format csv \
  -d "$out/fetch" -o run -- python3 -u bench.py --steps 1 --warmup 0 --cpu-seconds 1 "$@" > "$out/fetch.log" 2>&1
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "inflate_(block|tail)" --output-format csv \
  -d "$out/write" -o run -- python3 -u bench.py --steps 1 --warmup 0 --cpu-seconds 1 "$@" > "$out/write.log" 2>&1
python3 - "$out" "$summary" <<'PY'
import csv, glob, json, sys
out, summary = sys.argv[1], sys.argv[2]
vals = {}
for name in ("FETCH_SIZE", "WRITE_SIZE"):
    per = {}  # (kernel, dispatch) -> value (summed over the counter's instances)
    for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != name:
                continue
            k = "tail" if "inflate_tail" in r["Kernel_Name"] else "block" if "inflate_block" in r["Kernel_Name"] else None
            if k:
                key = (k, int(r["Dispatch_Id"]))
                per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    # one K2 launch = one block-kernel dispatch + one tail-kernel dispatch: the largest of each
    vals[name] = {k: max([v for (kk, _), v in per.items() if kk == k] or [0.0]) for k in ("block", "tail")}
fetch = {k: 2 * 1024 * v for k, v in vals["FETCH_SIZE"].items()}
write = {k: 1024 * v for k, v in vals["WRITE_SIZE"].items()}
res = {"kernel": "inflate_block_kernel + inflate_tail_kernel",
       "fetch_bytes_per_launch": sum(fetch.values()), "write_bytes_per_launch": sum(write.values()),
       "per_kernel_fetch_bytes": fetch, "per_kernel_write_bytes": write,
       "correction": "FETCH_SIZE x2 (gfx950: 64 B tallied per 128-B request), KiB -> bytes",
       "raw_FETCH_SIZE_KiB": vals["FETCH_SIZE"], "raw_WRITE_SIZE_KiB": vals["WRITE_SIZE"]}
res["traffic_bytes_per_launch"] = sum(fetch.values()) + sum(write.values())
json.dump(res, open(summary, "w"), indent=1)
print(json.dumps(res))
PY
