#!/bin/bash
# gemm2wg: parity tests, then isolated rates against the 256x256 kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm2wg_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03i_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r03i_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_gemm_2wg.py 2>&1 | grep -v amdgpu.ids
