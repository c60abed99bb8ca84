#!/bin/bash
# GELU forward in the A&S erfc form (ablibs/libgelu.so) and the GELU-free ceiling of the FFN-up
# epilogue (ablibs/libag.so, diagnostic): full GPU suite under the candidate, FFN-up / LN rates,
# step A/B vs in-tree
set -o pipefail
NEW=$PWD/ablibs/libgelu.so
mkdir -p gpurun_out
NRSE_LIB_PATH=$NEW timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/y_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/y_tests.log; exit 1; }
tail -1 gpurun_out/y_tests.log
for i in 1 2; do for l in "" $PWD/ablibs/libag.so $NEW; do
  echo -n "[${l:-in-tree}] "; NRSE_LIB_PATH=$l timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep ffn1 || exit 1
done; done
for l in "" $NEW; do echo "[${l:-in-tree}]"; NRSE_LIB_PATH=$l timeout -k 10 200 python -u tools/bench_ln.py 2>&1 | grep -E "fwd" || exit 1; done
run() { timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for i in 1 2; do
  echo -n "in-tree "; run || exit 1
  echo -n "gelu    "; NRSE_LIB_PATH=$NEW run || exit 1
done
