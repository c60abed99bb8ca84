#!/bin/bash
# r04 session 2: parity tests touched by the gate / LN change (kernels, engine, determinism),
# then the default bench with the gate read-modify-write form (NRSE_GATE_INTO_LN=0) and without, alternated.
# Usage: bash tools/gpu_r04e.sh
set -o pipefail
BASE=$1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_determinism_gpu.py tests/test_bf16_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/e_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/e_tests.log; exit 1; }
tail -1 gpurun_out/e_tests.log
bash tools/ab_env.sh "NRSE_GATE_INTO_LN=0" "-"
