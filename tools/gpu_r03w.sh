#!/bin/bash
# dK/dV kernel: diagonal fold without its own barrier (double-buffered staging, two bias copies):
# full GPU suite on the in-tree library, isolated attention and step vs ablibs/libnrse_old.so
set -o pipefail
OLD=$PWD/ablibs/libnrse_old.so
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/w_tests.log; exit 1; }
tail -1 gpurun_out/w_tests.log
for i in 1 2; do for lib in "$OLD" ""; do
  echo "== attn [${lib:-in-tree}]"; NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids || exit 1
done; done
run() { timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for i in 1 2; do
  echo -n "old     "; NRSE_LIB_PATH=$OLD run || exit 1
  echo -n "in-tree "; run || exit 1
done
