#!/bin/bash
# rocprof of the bench with the target view serialised onto the main stream (clean per-kernel times)
set -o pipefail
TAG=${1:-serial}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NRSE_SERIAL_TARGET=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
grep '"metric"' gpurun_out/${TAG}_bench.log | cut -c1-200
python tools/prof_summary.py gpurun_out/${TAG}_prof/run_kernel_stats.csv 7 40
