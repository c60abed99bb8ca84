#!/bin/bash
# gemm256 loop with balanced LDS reads (B-lo of t+1 read in phase 3 of t) vs the previous build
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
echo "-- stamps"
NRSE_LIB_PATH=$PWD/ablibs/libnrse_st.so timeout -k 10 200 python -u tools/diag_stamps.py 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
echo "-- product"
timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/bench_gemm_bwd.py 2>&1 | grep -v amdgpu.ids
echo "-- old"
NRSE_LIB_PATH=$PWD/ablibs/libnrse_old.so timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids
NRSE_LIB_PATH=$PWD/ablibs/libnrse_old.so timeout -k 10 200 python -u tools/bench_gemm_bwd.py 2>&1 | grep -v amdgpu.ids
done
