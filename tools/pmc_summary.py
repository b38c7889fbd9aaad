"""Utilisation roofline of K2 from a tools/pmc_inflate.sh counter summary (+ the traffic JSON).

usage: python3 tools/pmc_summary.py PMC_TXT TRAFFIC_JSON OUTPUT_BYTES_PER_DISPATCH OUT_JSON

Per kernel (block = inflate_block_kernel, tail = inflate_tail_kernel), from counters summed over
the run's dispatches (ratios are dispatch-count free):
  valu_issue_frac        SQ_INSTS_VALU / (SIMDs x cycles / 2): a wave64 VALU instruction takes a
                         SIMD-32 two cycles (MI355X_MICROARCH.md, 'Wave scheduling'); cycles =
                         GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs)
  valu_busy_quad_frac    SQ_ACTIVE_INST_VALU x 4 / (SIMDs x cycles): the same against the issue
                         cycles waves report (quad-cycles).  For these kernels SQ_ACTIVE_INST_VALU
                         equals SQ_INSTS_VALU: every VALU instruction holds a quad-cycle of its
                         SIMD's issue, so this, not valu_issue_frac, is the issue utilisation
                         (more waves per CU made K2 slower, fewer
                         VALU instructions made it faster)
  lds_busy_frac          SQ_LDS_IDX_ACTIVE / (CUs x cycles)
  lds_bank_conflict_frac SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  lds_unaligned_frac     SQ_LDS_UNALIGNED_STALL / SQ_LDS_IDX_ACTIVE
  valu_insts_per_output_byte  SQ_INSTS_VALU per decompressed byte (wave instructions)
  wait_frac              SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on waitcnt / barriers)
"""
import json
import sys

CUS, SIMDS = 256, 1024


def load(path):
    v = {}
    for line in open(path):
        if line.startswith("#") or not line.strip():
            continue
        p = line.split()
        v[(p[0], p[1])] = float(p[2])
    return v


def main():
    pmc, traffic, obytes, out = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    v = load(pmc)
    res = {"src": pmc, "output_bytes_per_dispatch": obytes, "kernels": {}}
    for k in ("block", "tail"):
        g = lambda n: v.get((k, n))  # noqa: E731
        if g("SQ_INSTS_VALU") is None:
            continue
        disp = 2  # tools/pmc_inflate.sh: two inflate dispatches per pass (the timing tool's runs)
        cyc = g("GRBM_GUI_ACTIVE") / 8
        r = {
            "cycles_per_dispatch": cyc / disp,
            "valu_issue_frac": g("SQ_INSTS_VALU") / (SIMDS * cyc / 2),
            "valu_busy_quad_frac": g("SQ_ACTIVE_INST_VALU") * 4 / (SIMDS * cyc),
            "lds_busy_frac": g("SQ_LDS_IDX_ACTIVE") / (CUS * cyc),
            "lds_bank_conflict_frac": g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"),
            "lds_unaligned_frac": g("SQ_LDS_UNALIGNED_STALL") / g("SQ_LDS_IDX_ACTIVE"),
            "valu_insts_per_output_byte": g("SQ_INSTS_VALU") / disp / obytes,
            "lds_insts_per_output_byte": g("SQ_INSTS_LDS") / disp / obytes,
            "wait_frac": g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"),
        }
        res["kernels"][k] = {a: round(b, 4) if b < 100 else round(b) for a, b in r.items()}
    try:
        t = json.load(open(traffic))
        res["traffic_bytes_per_launch"] = t.get("traffic_bytes_per_launch")
        res["traffic_src"] = traffic
    except OSError:
        pass
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
