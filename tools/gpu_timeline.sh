#!/bin/bash
# Kernel-trace timeline of the default bench step (tools/timeline.py: per-kernel exposed time, idle)
# Usage (on the GPU box): bash tools/gpu_timeline.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-tl}; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_trace -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-north-star "$@" > gpurun_out/${TAG}_trace.log 2>&1 || { tail -30 gpurun_out/${TAG}_trace.log; exit 1; }
python tools/timeline.py gpurun_out/${TAG}_trace/run_kernel_trace.csv 4 > gpurun_out/${TAG}_timeline.txt
head -45 gpurun_out/${TAG}_timeline.txt
rm -f gpurun_out/${TAG}_trace/run_kernel_trace.csv
