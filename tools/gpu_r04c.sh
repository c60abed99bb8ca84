#!/bin/bash
# r04 (session 2): parity tests of the touched kernels, isolated GEMM / conv0 rates under the
# baseline library and the in-tree one, then the default bench alternated twice on the same box.
# Usage (on the GPU box): bash tools/gpu_r04c.sh BASE_SO "pytest-args"
set -o pipefail
BASE=$1; TESTS=$2
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > gpurun_out/c_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c_tests.log; exit 1; }
  tail -1 gpurun_out/c_tests.log
fi
for lib in "$BASE" ""; do
  echo "== kernels [${lib:-in-tree}]"
  NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids || exit 1
  NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_gemm_bwd.py 2>&1 | grep -v amdgpu.ids || exit 1
  NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_ln.py 2>&1 | grep conv0 || exit 1
done
bash tools/ab_env.sh "NRSE_LIB_PATH=$BASE" "-"
