#!/bin/bash
# conv0 forward variants: parity tests, isolated timings under the baseline / in-tree libraries
# (twice), then the default bench alternated. Usage: bash tools/gpu_r04i.sh BASE_SO
set -o pipefail
BASE=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "conv0 or split3" -x -q --timeout 300 --timeout-method thread > gpurun_out/i_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/i_tests.log; exit 1; }
tail -1 gpurun_out/i_tests.log
for i in 1 2; do
  for lib in "$BASE" ""; do
    echo "== [${lib:-in-tree}]"
    NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_ln.py 2>&1 | grep "conv0 fwd" || exit 1
  done
done
bash tools/ab_env.sh "NRSE_LIB_PATH=$BASE" "-"
