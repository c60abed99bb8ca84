"""Per-kernel averages of rocprofv3 --pmc passes (counter_collection.csv) with derived ratios:
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs * 4 SIMDs) -- the
fraction of SIMD-cycles whose matrix pipe is busy --, the effective clock GRBM_GUI_ACTIVE / 8 /
duration, wait / issue fractions of the wave cycles, LDS bank-conflict share, L2 hit rate."""
import collections
import csv
import glob
import json
import os
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            key = (short, r.get("Grid_Size", ""), r.get("Workgroup_Size", ""))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if "End_Timestamp" in r and "Start_Timestamp" in r:
                dur[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {}
for key, cs in acc.items():
    m = {k: sum(v) / len(v) for k, v in cs.items()}
    row = dict(m)
    gui = m.get("GRBM_GUI_ACTIVE")
    if gui:
        simd_cycles = gui / 8 * 256 * 4
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            row["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
        if dur.get(key):
            row["eff_clock_ghz"] = gui / 8 / (sum(dur[key]) / len(dur[key]))
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in m:
                row[k.lower() + "_frac"] = m[k] / wc
    if m.get("SQ_LDS_IDX_ACTIVE"):
        row["lds_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"]
    if "TCC_HIT_sum" in m:
        row["l2_hit"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m.get("TCC_MISS_sum", 0))
    out[" ".join(k for k in key if k)] = row
for k, row in sorted(out.items(), key=lambda kv: kv[0]):
    if "at::native" in k:
        continue
    keys = ("mfma_busy", "eff_clock_ghz", "sq_wait_any_frac", "sq_wait_inst_any_frac", "sq_active_inst_any_frac",
            "lds_conflict_frac", "l2_hit")
    print(k[:80], {x: round(row[x], 3) for x in keys if x in row})
json.dump(out, open(os.path.join(sys.argv[1], "..", os.path.basename(sys.argv[1].rstrip("/")) + "_table.json"), "w"),
          indent=1)
