#!/bin/bash
# Same-box A/B of the in-tree library against a baseline build (NRSE_LIB_PATH), after the given
# parity tests pass on the in-tree one: isolated forward GEMMs + attention, then the default bench,
# alternated twice. Usage (on the GPU box): bash tools/gpu_ab2.sh TAG BASE_SO "tests/a.py ..."
set -o pipefail
TAG=$1; BASE=$2; TESTS=$3
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  tail -2 gpurun_out/${TAG}_tests.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
fi
for i in 1 2; do
  for lib in "$BASE" ""; do
    echo "== [${lib:-in-tree}]"
    NRSE_LIB_PATH=$lib timeout -k 10 180 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids || exit 1
    NRSE_LIB_PATH=$lib timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
for i in 1 2; do
  for lib in "$BASE" ""; do
    NRSE_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.err || { tail -20 gpurun_out/${TAG}_b.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_b.json')); print('bench [${lib:-in-tree}]', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
  done
done
