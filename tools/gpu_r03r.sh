#!/bin/bash
set -o pipefail
echo "-- attn product"; timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids
echo "-- attn bwd_q templated"; NRSE_LIB_PATH=$PWD/ablibs/libnrse_bq.so timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids
echo "-- attn product"; timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids
echo "-- attn bwd_q templated"; NRSE_LIB_PATH=$PWD/ablibs/libnrse_bq.so timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids
bash tools/gpu_ab_step.sh
