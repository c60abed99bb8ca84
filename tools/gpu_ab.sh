#!/bin/bash
# Same-box A/B driver (on the GPU box): parity tests on the in-tree build, isolated kernel
# microbenchmarks under each variant (alternated twice), then the default bench under each variant
# (tools/ab_env.sh, two passes).
#   bash tools/gpu_ab.sh "PYTEST_ARGS" "MICRO_SCRIPTS" VARIANT_A VARIANT_B ...
# PYTEST_ARGS: e.g. "tests/test_kernels_gpu.py -k conv0" ("" skips the tests); MICRO_SCRIPTS: e.g.
# "tools/bench_gemm_fwd.py tools/bench_ln.py" ("" skips them); each VARIANT is a space-separated
# list of VAR=value ("-" for none), e.g. "NRSE_LIB_PATH=noise-robust-speech-embedding_amd/ablib/base.so"
# or "NRSE_GATE_INTO_LN=0". (Session-2 r04 one-off scripts gpu_r04c..i were this driver's cases.)
set -o pipefail
TESTS=$1; MICRO=$2; shift 2
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
if [ -n "$MICRO" ]; then
  for pass in 1 2; do
    for v in "$@"; do
      envs=""; [ "$v" != "-" ] && envs="$v"
      for m in $MICRO; do
        echo "== pass $pass [$v] $m"
        env $envs timeout -k 10 240 python -u $m 2>&1 | grep -v amdgpu.ids || exit 1
      done
    done
  done
fi
bash tools/ab_env.sh "$@"
