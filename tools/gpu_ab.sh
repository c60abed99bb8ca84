#!/bin/bash
# A/B of a diagnostic build (ablibs/libnrse_$1.so) against the in-tree library on the isolated
# step GEMM shapes, interleaved twice; then the per-barrier timeline of the phase-stamp build.
set -o pipefail
V=$1
for i in 1 2; do
echo "-- tree"; ROWS=224 timeout -k 10 300 python -u tools/bench_gemm_bm.py 2>&1 | grep -v amdgpu.ids
echo "-- $V"; NRSE_LIB_PATH=$PWD/ablibs/libnrse_$V.so ROWS=224 timeout -k 10 300 python -u tools/bench_gemm_bm.py 2>&1 | grep -v amdgpu.ids
done
if [ -f ablibs/libnrse_phases.so ]; then NRSE_LIB_PATH=$PWD/ablibs/libnrse_phases.so timeout -k 10 120 python -u tools/diag_phases.py 2>&1 | grep -v amdgpu.ids; fi
