#!/bin/bash
# r06 quick check of the LDS-DMA drain fixes: the GEMM / attention / determinism / engine tests,
# the isolated attention and GEMM benches, and the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm256_gpu.py tests/test_fp8_gpu.py tests/test_attention_gpu.py tests/test_kernels_gpu.py tests/test_determinism_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_attn_q.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06_attn_q.log; exit 1; }
tail -1 gpurun_out/r06_attn_q.log
for pass in 1 2; do timeout -k 10 200 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06_bench_q.json 2> gpurun_out/r06_bench_q.err || { tail -20 gpurun_out/r06_bench_q.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r06_bench_q.json')); print(d['value'], d['ms_per_step'], d.get('north_star_mode',{}).get('value'), d['roofline']['achieved'], d['roofline']['frac'])"
