#!/bin/bash
# gemm256 epilogue: bias fetched before the main loop + direct f32 stores, vs the previous build
set -o pipefail
echo "-- stamps"
NRSE_LIB_PATH=$PWD/ablibs/libnrse_st.so timeout -k 10 200 python -u tools/diag_stamps.py 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
echo "-- product"
GENS=0 timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids
echo "-- old"
GENS=0 NRSE_LIB_PATH=$PWD/ablibs/libnrse_old.so timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids
done
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
