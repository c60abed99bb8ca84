#!/bin/bash
# deterministic reductions: new tests first, then the whole GPU suite, the bench and a GEMM A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_determinism_gpu.py tests/test_gemm256_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03m_det.log 2>&1; rc=$?
tail -12 gpurun_out/r03m_det.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_round.sh r03m || exit 1
echo "-- gemm A/B"
timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids
NRSE_LIB_PATH=$PWD/ablibs/libnrse_old.so timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/bench_gemm_bwd.py 2>&1 | grep -v amdgpu.ids
