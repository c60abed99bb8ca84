#!/bin/bash
# One GPU iteration: parity tests, then a profiled short bench. Usage (on the GPU box, via gpurun):
#   bash tools/gpu_iter.sh TAG "pytest-files" [bench-args]
set -o pipefail
TAG=$1; TESTS=$2; shift 2
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -m pytest $TESTS -x -q > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
grep '"metric"' gpurun_out/${TAG}_bench.log | cut -c1-400
python tools/prof_summary.py gpurun_out/${TAG}_prof/run_kernel_stats.csv 7 25
