#!/bin/bash
# Same-box A/B of environment settings on the default bench: bash tools/ab_env.sh "ENV_A" "ENV_B" ...
# (each argument is a space-separated list of VAR=value, "-" for none); two passes in order.
set -o pipefail
mkdir -p gpurun_out
for pass in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    envs=""; [ "$e" != "-" ] && envs="$e"
    out=$(env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline 2> gpurun_out/ab_err_$i.log) || { echo "run $i failed"; tail -20 gpurun_out/ab_err_$i.log; exit 1; }
    echo "pass $pass [$e]: $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
