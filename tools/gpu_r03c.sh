#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for v in stamps abl9 abl10; do
echo "== $v"
NRSE_LIB_PATH=$PWD/ablibs/libnrse_$v.so SHAPES=short timeout -k 10 200 python -u tools/diag_stamps.py 2>&1 | grep -v amdgpu.ids
done | tee gpurun_out/r03c_stamps.txt
