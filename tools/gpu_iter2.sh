#!/bin/bash
# one GPU iteration: the given test files, isolated attention kernels, the default bench twice.
# Usage (on the GPU box): bash tools/gpu_iter2.sh TAG "tests/a.py tests/b.py"
set -o pipefail
TAG=$1; TESTS=$2
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/${TAG}_tests.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
fi
timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench$i.json 2> gpurun_out/${TAG}_bench$i.err || { tail -20 gpurun_out/${TAG}_bench$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench$i.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done
