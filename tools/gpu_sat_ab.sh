#!/bin/bash
# r06 A/B: the saturation count's fast path (default) against the exact count on every call
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_saturation_gpu.py tests/test_fp8_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_sat_ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06_sat_ab_tests.log; exit 1; }
tail -1 gpurun_out/r06_sat_ab_tests.log
for pass in 1 2; do
  for v in "" oldsat; do
    if [ -n "$v" ]; then export NRSE_LIB_PATH=noise-robust-speech-embedding_amd/ablib/$v.so; else unset NRSE_LIB_PATH; fi
    echo "== pass $pass [$v]"
    timeout -k 10 200 python -u tools/bench_conv0.py 2>&1 | grep -v amdgpu.ids || exit 1
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > /tmp/b.json 2> /tmp/b.err || { tail -20 /tmp/b.err; exit 1; }
    python -c "import json; d=json.load(open('/tmp/b.json')); print('bench', d['value'], d['ms_per_step'], 'bf16sw', d.get('north_star_mode',{}).get('value'))"
  done
done
