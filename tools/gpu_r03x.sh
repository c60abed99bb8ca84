#!/bin/bash
# GEMM tile-group depth (GM M-tiles per group of the XCD-aware order): isolated forward / backward
# GEMM rates and the step for GM = 4, 16, 32 (ablibs/libgm*.so) vs the in-tree GM = 8
set -o pipefail
mkdir -p gpurun_out
for v in 8 4 16 32; do
  lib=""; [ $v != 8 ] && lib=$PWD/ablibs/libgm$v.so
  echo "== GM=$v fwd"; NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== GM=$v bwd"; NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_gemm_bwd.py 2>&1 | grep -v amdgpu.ids || exit 1
done
run() { timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])"; }
for i in 1 2; do for v in 8 4 16 32; do
  lib=""; [ $v != 8 ] && lib=$PWD/ablibs/libgm$v.so
  echo -n "GM=$v step "; NRSE_LIB_PATH=$lib run || exit 1
done; done
