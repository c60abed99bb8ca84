#!/bin/bash
# bf16 GEMM epilogue stored from registers after permlane16 swaps vs the LDS-staged rows
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
for i in 1 2; do
echo "-- product"
timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids
echo "-- old"
NRSE_LIB_PATH=$PWD/ablibs/libnrse_old.so timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids
done
echo "-- step product / old / product"
timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
NRSE_LIB_PATH=$PWD/ablibs/libnrse_old.so timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
