#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm256_gpu.py tests/test_gemm_gpu.py tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03g_tests.log 2>&1 || { tail -30 gpurun_out/r03g_tests.log; exit 1; }
tail -1 gpurun_out/r03g_tests.log
bash tools/gpu_roofline.sh r03g
