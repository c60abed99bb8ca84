#!/bin/bash
# full GPU suite, then the N = 2 launch path rehearsed with two ranks sharing the card over gloo
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r04b_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04b_tests.log | head -20; exit $rc; }
NRSE_SHARE_DEVICE=1 NRSE_DDP_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04b_2rank.json 2> gpurun_out/r04b_2rank.err || { tail -30 gpurun_out/r04b_2rank.err; exit 1; }
grep '^{' gpurun_out/r04b_2rank.json > gpurun_out/r04b_2rank_line.json && python -c "import json; d=json.load(open('gpurun_out/r04b_2rank_line.json')); print(d['value'], d['ms_per_step'], d['ddp'])"
