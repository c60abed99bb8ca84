#!/bin/bash
# r04 session 2: attention parity tests, isolated attention under the baseline / in-tree
# libraries (alternated), the host-gap diagnostic. Usage: bash tools/gpu_r04d.sh BASE_SO
set -o pipefail
BASE=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/d_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/d_tests.log; exit 1; }
tail -1 gpurun_out/d_tests.log
for i in 1 2; do
  for lib in "$BASE" ""; do
    echo "== attn [${lib:-in-tree}]"
    NRSE_LIB_PATH=$lib timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
timeout -k 10 300 python -u tools/diag_hostgap.py > gpurun_out/d_hostgap.txt 2>&1 || { tail -20 gpurun_out/d_hostgap.txt; exit 1; }
cat gpurun_out/d_hostgap.txt
