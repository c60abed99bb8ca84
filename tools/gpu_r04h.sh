#!/bin/bash
# r04 session 2: rows_reduce tests + the determinism suite, then the default bench under the
# baseline library and the in-tree one alternated. Usage: bash tools/gpu_r04h.sh BASE_SO
set -o pipefail
BASE=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_determinism_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/h_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/h_tests.log; exit 1; }
tail -1 gpurun_out/h_tests.log
bash tools/ab_env.sh "NRSE_LIB_PATH=$BASE" "-"
