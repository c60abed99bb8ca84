#!/bin/bash
# Same-box comparison of library variants (NRSE_LIB_PATH; "-" = the in-tree build): isolated
# forward GEMMs and attention, then the default bench, alternated twice.
# Usage (on the GPU box): bash tools/gpu_abn.sh TAG "libA.so - libB.so ..."
set -o pipefail
TAG=$1; LIBS=$2
mkdir -p gpurun_out
for i in 1 2; do
  for lib in $LIBS; do
    [ "$lib" = "-" ] && lib=""
    echo "== [${lib:-in-tree}]"
    NRSE_LIB_PATH=$lib timeout -k 10 180 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids || exit 1
    NRSE_LIB_PATH=$lib timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
for i in 1 2; do
  for lib in $LIBS; do
    [ "$lib" = "-" ] && lib=""
    NRSE_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.err || { tail -20 gpurun_out/${TAG}_b.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_b.json')); print('bench [${lib:-in-tree}]', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
  done
done
