#!/bin/bash
# attention forward with the transposed PV MFMA (own-row rescale, 8-byte ctx stores) vs previous
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
for i in 1 2; do
echo "-- product"; timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids
echo "-- old"; NRSE_LIB_PATH=$PWD/ablibs/libnrse_old.so timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids
done
