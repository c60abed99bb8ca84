#!/bin/bash
# Same-box A/B of a baseline library build against the in-tree one:
#   bash tools/ab_lib.sh BASE_SO "pytest-files"
# parity tests on the in-tree library, the isolated LN / conv0 kernels under both, then the
# default bench alternated twice.
set -o pipefail
BASE=$1; TESTS=$2
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for lib in "$BASE" ""; do
  echo "== kernels [${lib:-in-tree}]"
  NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_ln.py 2>&1 | grep conv0 || exit 1
done
bash tools/ab_env.sh "NRSE_LIB_PATH=$BASE" "-"
