#!/bin/bash
# Final-tree check (r06): the full GPU suite, smoke(), the default bench line with the CPU baseline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 400 --timeout-method thread > gpurun_out/r06_final_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06_final_tests.log; exit 1; }
tail -1 gpurun_out/r06_final_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_final_smoke.log 2>&1 || { tail -20 gpurun_out/r06_final_smoke.log; exit 1; }
tail -2 gpurun_out/r06_final_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r06_final_bench.json 2> gpurun_out/r06_final_bench.err || { tail -30 gpurun_out/r06_final_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r06_final_bench.json')); print(d['value'], d['ms_per_step'], d.get('north_star_mode',{}).get('value'), d['roofline']['frac'], d['cpu_baseline']['value'])"
