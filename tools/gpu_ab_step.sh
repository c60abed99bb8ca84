#!/bin/bash
# same-box step A/B: the in-tree library vs ablibs/libnrse_old.so, alternating
set -o pipefail
run() { timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for i in 1 2; do
echo -n "product "; run
echo -n "old     "; NRSE_LIB_PATH=$PWD/ablibs/libnrse_old.so run
done
