#!/bin/bash
# Full GPU pass (via gpurun): parity tests, default bench (with CPU baseline), rocprof stats.
# Usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_profbench.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/${TAG}_profbench.log; exit 1; }
grep '"metric"' gpurun_out/${TAG}_profbench.log | cut -c1-300
python tools/prof_summary.py gpurun_out/${TAG}_prof/run_kernel_stats.csv 7 25
