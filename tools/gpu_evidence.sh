#!/bin/bash
# Round-4 evidence on one box: SQ/GRBM/TCC counter passes of the isolated hot kernels
# (tools/pmc_sq.sh), HBM traffic of the step's GEMMs (tools/pmc_gemm.sh), the default bench line
# (with the CPU baseline), and its serial rocprofv3 kernel-trace summary.
# Usage (on the GPU box): bash tools/gpu_evidence.sh TAG
# (gpurun merges gpurun_out/ back: copy ${TAG}_sq_p1_table.json / ${TAG}_traffic.json into profiles/
# as the round's SQ table / GEMM traffic files, which bench.py reads)
set -o pipefail
TAG=${1:-r04e}
mkdir -p gpurun_out
bash tools/pmc_sq.sh ${TAG}_sq all > gpurun_out/${TAG}_sq.txt 2>&1 || { tail -20 gpurun_out/${TAG}_sq.txt; exit 1; }
grep -E "gemm256|attn" gpurun_out/${TAG}_sq.txt | head -20
bash tools/pmc_gemm.sh ${TAG} || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline'], d['cpu_baseline'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NRSE_SERIAL_TARGET=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_serial -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-north-star > gpurun_out/${TAG}_serial.log 2>&1 || { tail -30 gpurun_out/${TAG}_serial.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_serial/run_kernel_stats.csv 9 12
