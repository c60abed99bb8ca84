#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm256_gpu.py tests/test_gemm_gpu.py tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03b_tests.log 2>&1 || { tail -30 gpurun_out/r03b_tests.log; exit 1; }
tail -2 gpurun_out/r03b_tests.log
timeout -k 10 300 python -u tools/bench_gemm_bm.py 2>&1 | tee gpurun_out/gbm_bench.txt
echo "--- attention new"; timeout -k 10 120 python -u tools/bench_attn.py
echo "--- attention old"; NRSE_LIB_PATH=$PWD/ablibs/libnrse_attold.so timeout -k 10 120 python -u tools/bench_attn.py
echo "--- attention new"; timeout -k 10 120 python -u tools/bench_attn.py
