#!/bin/bash
# In-step kernel trace of the default bench (streams overlapped as in the timed steps) and its
# exposed-time view (tools/timeline.py), plus the per-kernel stats. Usage: bash tools/gpu_timeline.sh TAG
set -o pipefail
TAG=${1:-tl}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-north-star > gpurun_out/${TAG}_trace.log 2>&1 || { tail -30 gpurun_out/${TAG}_trace.log; exit 1; }
python tools/timeline.py gpurun_out/${TAG}_trace/run_kernel_trace.csv 4 > gpurun_out/${TAG}_timeline.txt
head -45 gpurun_out/${TAG}_timeline.txt
python tools/prof_summary.py gpurun_out/${TAG}_trace/run_kernel_stats.csv 9 30 > gpurun_out/${TAG}_stats.txt
rm -f gpurun_out/${TAG}_trace/run_kernel_trace.csv.gz
