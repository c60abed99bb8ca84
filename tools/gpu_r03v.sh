#!/bin/bash
# shared-exponential GELU': full GPU suite on the in-tree library, isolated LN / conv0 / GEMM
# backward and the step vs ablibs/libnrse_old.so (HEAD), alternating
set -o pipefail
OLD=$PWD/ablibs/libnrse_old.so
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/v_tests.log; exit 1; }
tail -1 gpurun_out/v_tests.log
for lib in "$OLD" ""; do
  echo "== ln/conv0 [${lib:-in-tree}]"; NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_ln.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== bwd [${lib:-in-tree}]"; NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_gemm_bwd.py 2>&1 | grep -v amdgpu.ids || exit 1
done
run() { timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for i in 1 2; do
  echo -n "old     "; NRSE_LIB_PATH=$OLD run || exit 1
  echo -n "in-tree "; run || exit 1
done
