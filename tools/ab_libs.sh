#!/bin/bash
# Isolated kernel times (tools/bench_ln.py lines matching PATTERN) under each library variant in
# noise-robust-speech-embedding_amd/ablib/, after TESTS pass on the in-tree library.
#   bash tools/ab_libs.sh PATTERN "pytest-args"
set -o pipefail
PAT=$1; TESTS=$2
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/abl_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/abl_tests.log; exit 1; }
  tail -1 gpurun_out/abl_tests.log
fi
for lib in noise-robust-speech-embedding_amd/ablib/*.so ""; do
  echo "== ${lib:-in-tree}"
  NRSE_LIB_PATH=$lib timeout -k 10 120 python -u tools/bench_ln.py 2>&1 | grep "$PAT" || exit 1
done
