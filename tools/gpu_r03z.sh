#!/bin/bash
# packed-FP32 GELU in the FFN-up register epilogue (ablibs/libpk.so) vs in-tree: step A/B
set -o pipefail
run() { timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for i in 1 2 3; do
  echo -n "in-tree "; run || exit 1
  echo -n "pk      "; NRSE_LIB_PATH=$PWD/ablibs/libpk.so run || exit 1
done
