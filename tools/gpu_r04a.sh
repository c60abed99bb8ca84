#!/bin/bash
# r04 iteration: split-weight tests + Large parity (bf16sw, bf16 heads), then bf16 / bf16sw benches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_large_gpu.py \
  -k "split or bf16sw or heads" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|bf16sw_|bf16_heads" gpurun_out/r04a_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
for d in bf16 bf16sw bf16; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --dtype $d > gpurun_out/r04a_bench_$d.json 2> gpurun_out/r04a_bench_$d.err || { tail -20 gpurun_out/r04a_bench_$d.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r04a_bench_$d.json')); print('$d', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done
