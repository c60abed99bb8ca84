#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gbm_tests.log 2>&1 || { tail -30 gpurun_out/gbm_tests.log; exit 1; }
tail -2 gpurun_out/gbm_tests.log
timeout -k 10 300 python -u tools/bench_gemm_bm.py 2>&1 | tee gpurun_out/gbm_bench.txt
