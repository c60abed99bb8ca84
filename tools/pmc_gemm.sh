#!/bin/bash
# HBM traffic of the GEMM family in the bench step (MI355X_MICROARCH.md HBM/rocprofv3 recipe):
# one rocprofv3 --pmc pass per counter (FETCH_SIZE, WRITE_SIZE), bench kept short, GEMM kernels
# only. Usage (on the GPU box): bash tools/pmc_gemm.sh TAG  -> gpurun_out/TAG_traffic.json
set -o pipefail
TAG=${1:-pmc}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm --output-format csv -d gpurun_out/${TAG}_fetch -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-north-star > gpurun_out/${TAG}_fetch.log 2>&1 || { tail -20 gpurun_out/${TAG}_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex gemm --output-format csv -d gpurun_out/${TAG}_write -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-north-star > gpurun_out/${TAG}_write.log 2>&1 || { tail -20 gpurun_out/${TAG}_write.log; exit 1; }
python tools/pmc_summary.py gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write > gpurun_out/${TAG}_traffic.json
grep family gpurun_out/${TAG}_traffic.json
