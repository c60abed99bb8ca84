#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py tests/test_gemm_gpu.py -x -q --timeout 100 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1 || { tail -30 gpurun_out/r03e_tests.log; exit 1; }
tail -1 gpurun_out/r03e_tests.log
timeout -k 10 300 python -u tools/bench_gemm_bm.py 2>&1 | grep -v amdgpu.ids
NRSE_LIB_PATH=$PWD/ablibs/libnrse_stamps.so timeout -k 10 200 python -u tools/diag_stamps.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 100 python -u tools/bench_gemm_stagger.py 2>&1 | grep -v amdgpu.ids
