#!/bin/bash
# gemm2wg diagnostics: product vs no in-loop DMA (d1), no vmcnt wait (d2), no barrier (d3)
set -o pipefail
timeout -k 10 200 python -u tools/bench_gemm_2wg.py 2>&1 | grep -v amdgpu.ids
for d in 1 2 3; do
echo "-- d$d"
GENS=5 NRSE_LIB_PATH=$PWD/ablibs/libnrse_d$d.so timeout -k 10 200 python -u tools/bench_gemm_2wg.py 2>&1 | grep -v amdgpu.ids
done
