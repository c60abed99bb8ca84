#!/bin/bash
# LDS counters of the GEMM layouts (TT forward, TF dgrad, FF weight gradient) on isolated step
# shapes: one rocprofv3 --pmc pass, SQ counters only. -> gpurun_out/lds_pmc/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex gemm256 --output-format csv -d gpurun_out/lds_pmc -o run -- python3 tools/bench_gemm_bwd.py > gpurun_out/lds_pmc.log 2>&1 || { tail -20 gpurun_out/lds_pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/lds_pmc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].split("::")[-1] + f" grid={r.get('Grid_Size', '?')}"
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    c = n[(k, "SQ_WAVE_CYCLES")] or 1
    print(k, " ".join(f"{name}={v / c:.3g}" for name, v in sorted(d.items())))
PY
