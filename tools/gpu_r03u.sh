#!/bin/bash
# dK/dV diagonal-sum ablations (diagnostic builds ablibs/libabl{1,2,3}.so: 1 no fold, 2 no DPP
# accumulation, 3 no partial-row store) vs in-tree: per-kernel durations from rocprofv3 stats
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1 2 3; do
  lib=""; [ $v -gt 0 ] && lib=$PWD/ablibs/libabl$v.so
  NRSE_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u$v -o run -- python tools/bench_attn.py > gpurun_out/u$v.log 2>&1 || { echo "prof $v failed"; tail -5 gpurun_out/u$v.log; exit 1; }
  echo "== variant $v"; grep -v amdgpu.ids gpurun_out/u$v.log | grep "p=" 
  python - <<PY
import csv
for r in csv.DictReader(open("gpurun_out/u$v/run_kernel_stats.csv")):
    if "attn" in r["Name"] or "rows_reduce" in r["Name"]:
        print(f'  {float(r["AverageNs"])/1e3:8.1f} us  n={r["Calls"]:>4}  {r["Name"][:70]}')
PY
done
