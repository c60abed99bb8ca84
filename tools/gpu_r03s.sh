#!/bin/bash
# 208-row GEMM tiles + attention forward lazy rescale: parity under the candidate libraries,
# isolated GEMM / attention rates and the step, candidates vs in-tree, alternating.
set -o pipefail
L208=$PWD/ablibs/libnrse_208.so
NEW=$PWD/ablibs/libnrse_new.so
mkdir -p gpurun_out
NRSE_LIB_PATH=$NEW timeout -k 10 500 python -u -m pytest tests/test_gemm256_gpu.py tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/s_tests.log; exit 1; }
tail -1 gpurun_out/s_tests.log
for lib in "" "$NEW"; do
  echo "== attn [${lib:-in-tree}]"; NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== fwd [${lib:-in-tree}]"; NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== bwd [${lib:-in-tree}]"; NRSE_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_gemm_bwd.py 2>&1 | grep -v amdgpu.ids || exit 1
done
run() { timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])"; }
for i in 1 2; do
  echo -n "in-tree "; run || exit 1
  echo -n "208     "; NRSE_LIB_PATH=$L208 run || exit 1
  echo -n "new     "; NRSE_LIB_PATH=$NEW run || exit 1
done
