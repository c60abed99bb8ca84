#!/bin/bash
# GEMM gen-3 stamped ablations (diag_libs_st*.so built locally): per-phase cycles per variant
set -o pipefail
mkdir -p gpurun_out
for v in "" 1 2 3 4 5 7 8; do
  echo "== variant '$v'" >> gpurun_out/ablate.log
  NRSE_LIB_PATH=$PWD/noise-robust-speech-embedding_amd/diag_libs_st$v.so timeout -k 10 120 python -u tools/diag_stamps.py >> gpurun_out/ablate.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/ablate.log
