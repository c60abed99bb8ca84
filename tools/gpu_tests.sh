#!/bin/bash
# GPU test subset (via gpurun): bash tools/gpu_tests.sh TAG "tests/a.py tests/b.py ..."
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $@ -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -60
exit $rc
