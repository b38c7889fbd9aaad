"""Dev tool: turn a tools/gpu_evidence.sh output directory into the committed profile summaries.

usage: python3 tools/evidence_summary.py EVDIR TAG "kernel description"
writes profiles/TAG_rocprof_summary.txt, TAG_kernel_stats.csv, TAG_inflate_traffic_pmc.json,
TAG_prof_bench.json and TAG_inflate_pmc.txt (raw counters + derived ratios)."""
import csv
import glob
import json
import os
import shutil
import sys

ev, tag, desc = sys.argv[1], sys.argv[2], sys.argv[3]
P = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles")
shutil.copy(os.path.join(ev, "kernel_stats.csv"), os.path.join(P, f"{tag}_kernel_stats.csv"))
shutil.copy(os.path.join(ev, "traffic.json"), os.path.join(P, f"{tag}_inflate_traffic_pmc.json"))
shutil.copy(os.path.join(ev, "prof_bench.json"), os.path.join(P, f"{tag}_prof_bench.json"))
tr = glob.glob(os.path.join(ev, "prof", "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(tr)))
inf = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
       if "inflate_block" in r["Kernel_Name"]]
big = [x for x in inf if x > 10]
small = [x for x in inf if x <= 10]
bench = json.load(open(os.path.join(ev, "prof_bench.json")))
stats = list(csv.DictReader(open(os.path.join(ev, "kernel_stats.csv"))))
short = lambda n: n.replace("dq::(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]
others = ", ".join(f"{short(r['Name'])} {float(r['AverageNs']) / 1e6:.2f} ms" for r in stats[1:7])
traffic = json.load(open(os.path.join(ev, "traffic.json")))
alg = bench["roofline"]["alg_bytes_per_launch"]
with open(os.path.join(P, f"{tag}_rocprof_summary.txt"), "w") as f:
    f.write("# rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py --steps 3 --warmup 1 "
            "--cpu-seconds 1 --e2e 0 --intervals 0\n")
    f.write(f"# (tools/gpu_evidence.sh; MI355X, N = 1, 12.5 GB configs[2]-family file; {desc};\n")
    f.write(f"#  full table: profiles/{tag}_kernel_stats.csv; bench line of this run: profiles/{tag}_prof_bench.json)\n")
    f.write(f"# inflate_block_kernel<false,4,1>, whole-file launches: {len(big)} launches,\n")
    f.write("#   " + " ".join(f"{x:.3f}" for x in big) + f" ms -> average {sum(big) / len(big):.3f} ms"
            f"  (bench.py HIP events: {bench['roofline']['avg_launch_ms']} ms)\n")
    if small:
        f.write(f"#   plus {len(small)} {small[0]:.3f} ms launch (the header prefix read by bench's header broadcast)\n")
    f.write(f"# {others}\n")
    f.write(f"# PMC traffic of the same workload (tools/pmc_traffic.sh, two passes): profiles/{tag}_inflate_traffic_pmc.json\n")
    f.write(f"#   FETCH_SIZE x2 = {traffic['fetch_bytes_per_launch'] / 1e9:.2f} GB, WRITE_SIZE = "
            f"{traffic['write_bytes_per_launch'] / 1e9:.2f} GB, traffic {traffic['traffic_bytes_per_launch'] / 1e9:.2f} GB "
            f"per launch vs {alg / 1e9:.2f} GB algorithmic ({traffic['traffic_bytes_per_launch'] / alg:.3f} x)\n")
v = {}
for line in open(os.path.join(ev, "sq.log")):
    p = line.split()
    # "block NAME value ..." (tools/pmc_inflate.sh: per kernel); the derived lines use the block kernel
    if len(p) >= 3 and p[0] == "block" and p[1].isupper():
        v[p[1]] = float(p[2])
    elif len(p) >= 2 and p[0].isupper():
        v[p[0]] = float(p[1])
with open(os.path.join(P, f"{tag}_inflate_pmc.txt"), "w") as f:
    f.write(f"# inflate_block_kernel PMC counters, {desc}\n")
    f.write("# tools/pmc_inflate.sh: 5 rocprofv3 --pmc passes over tools/inflate_timing.py 2000000 "
            "(2 dispatches of ~10K BGZF blocks summed; MI355X)\n")
    f.write("# SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* are quad-cycles (MI355X_MICROARCH.md).\n")
    f.write(open(os.path.join(ev, "sq.log")).read())
    w = v["SQ_WAVES"]
    f.write(f"\n# derived (per dispatch): waves {w / 2:,.0f}; VALU insts/wave {v['SQ_INSTS_VALU'] / w / 1e3:.1f}K, "
            f"SALU {v['SQ_INSTS_SALU'] / w / 1e3:.1f}K, LDS {v['SQ_INSTS_LDS'] / w / 1e3:.2f}K\n")
    f.write(f"# VALU busy = ACTIVE_INST_VALU*4 / (1024 SIMDs * GRBM_GUI_ACTIVE/8 XCDs) = "
            f"{100 * v['SQ_ACTIVE_INST_VALU'] * 4 / (1024 * v['GRBM_GUI_ACTIVE'] / 8):.1f} %\n")
    wc = v["SQ_WAVE_CYCLES"]
    f.write(f"# wave-cycle split: WAIT_ANY {100 * v['SQ_WAIT_ANY'] / wc:.1f} %, ACTIVE_INST_ANY "
            f"{100 * v['SQ_ACTIVE_INST_ANY'] / wc:.1f} %, WAIT_INST_ANY {100 * v['SQ_WAIT_INST_ANY'] / wc:.1f} %\n")
    f.write(f"# LDS bank conflicts: {100 * v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE']:.1f} % of LDS-active cycles\n")
    f.write(f"# GRBM_GUI_ACTIVE {v['GRBM_GUI_ACTIVE']:.4g} (r2cl, end of round 2: 2.038e8; r3ab: 1.741e8)\n")
print(open(os.path.join(P, f"{tag}_rocprof_summary.txt")).read())
print(open(os.path.join(P, f"{tag}_inflate_pmc.txt")).read()[-600:])
