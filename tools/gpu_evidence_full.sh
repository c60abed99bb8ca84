#!/bin/bash
# Evidence on one box (r04 session 2, r05): the full GPU suite, the r04 evidence pass
# (tools/gpu_evidence.sh: SQ table, GEMM traffic, default bench with the CPU baseline, serial
# kernel stats), the conv0 counter pass and the in-step kernel stats.
# Usage (on the GPU box): bash tools/gpu_evidence_full.sh TAG
set -o pipefail
TAG=${1:-r04g}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
bash tools/gpu_evidence.sh ${TAG}e || exit 1
bash tools/pmc_sq.sh ${TAG}_c0 conv0 > gpurun_out/${TAG}_c0.txt 2>&1 || { tail -20 gpurun_out/${TAG}_c0.txt; exit 1; }
grep -E "conv0" gpurun_out/${TAG}_c0.txt | head
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_instep -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-north-star > gpurun_out/${TAG}_instep.log 2>&1 || { tail -30 gpurun_out/${TAG}_instep.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_instep/run_kernel_stats.csv 8 14
rm -f gpurun_out/${TAG}_instep/run_kernel_trace.csv gpurun_out/${TAG}e_serial/run_kernel_trace.csv
# the north-star mode's in-step kernel stats (bf16sw line)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_instep_sw -o run -- python bench.py --dtype bf16sw --steps 5 --warmup 2 --no-cpu-baseline --no-north-star > gpurun_out/${TAG}_instep_sw.log 2>&1 || { tail -30 gpurun_out/${TAG}_instep_sw.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_instep_sw/run_kernel_stats.csv 8 14
rm -f gpurun_out/${TAG}_instep_sw/run_kernel_trace.csv
