#!/bin/bash
# attention bias-copy bank swizzle: parity, isolated rates, PMC, step A/B vs in-tree
set -o pipefail
NEW=$PWD/ablibs/libnrse_swz.so
mkdir -p gpurun_out
NRSE_LIB_PATH=$NEW timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_tests.log; exit 1; }
tail -1 gpurun_out/t_tests.log
for i in 1 2; do for lib in "" "$NEW"; do
  echo "== attn [${lib:-in-tree}]"; NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids || exit 1
done; done
NRSE_LIB_PATH=$NEW bash tools/pmc_sq.sh r03_attn_swz attn || exit 1
run() { timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for i in 1 2; do
  echo -n "in-tree "; run || exit 1
  echo -n "swz     "; NRSE_LIB_PATH=$NEW run || exit 1
done
