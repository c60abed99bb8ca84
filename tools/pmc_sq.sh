#!/bin/bash
# SQ / GRBM / TCC counters of the hot kernels (tools/kernel_driver.py), one rocprofv3 --pmc pass
# per counter group (MI355X_MICROARCH.md: <= 8 SQ, 2 GRBM, 4 TCC per pass; no trace domains).
# Usage (on the GPU box): bash tools/pmc_sq.sh TAG [gemm|attn|all]
set -o pipefail
TAG=${1:-sq}; WHAT=${2:-all}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
P3="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python tools/kernel_driver.py $WHAT > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python tools/pmc_table.py gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2 gpurun_out/${TAG}_p3
