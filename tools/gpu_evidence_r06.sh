#!/bin/bash
# Round-6 evidence from the final tree, in two box calls (each under gpurun's 20-minute limit):
#   bash tools/gpu_evidence_r06.sh A   full GPU suite (-s: the parity tests' printed deviations),
#                                      the train_byol loop trace, the default bench line
#   bash tools/gpu_evidence_r06.sh B   tools/gpu_evidence.sh (SQ counter table, GEMM traffic, bench
#                                      with the CPU baseline, serial kernel stats), the conv0 counter
#                                      pass, the in-step kernel stats of the bf16 and bf16sw lines
set -o pipefail
PART=${1:-A}
mkdir -p gpurun_out
if [ "$PART" = A ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 400 --timeout-method thread > gpurun_out/r06_suite_final.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06_suite_final.log; exit 1; }
  tail -1 gpurun_out/r06_suite_final.log
  bash tools/trace_train_loop.sh r06_trainloop || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06_benchA.json 2> gpurun_out/r06_benchA.err || { tail -30 gpurun_out/r06_benchA.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r06_benchA.json')); print(d['value'], d['ms_per_step'], d.get('north_star_mode',{}).get('value'))"
else
  bash tools/gpu_evidence.sh r06e || exit 1
  bash tools/pmc_sq.sh r06_c0 conv0 > gpurun_out/r06_c0.txt 2>&1 || { tail -20 gpurun_out/r06_c0.txt; exit 1; }
  grep -E "conv0" gpurun_out/r06_c0.txt | head
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_instep -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-north-star > gpurun_out/r06_instep.log 2>&1 || { tail -30 gpurun_out/r06_instep.log; exit 1; }
  python tools/prof_summary.py gpurun_out/r06_instep/run_kernel_stats.csv 8 14
  rm -f gpurun_out/r06_instep/run_kernel_trace.csv gpurun_out/r06e_serial/run_kernel_trace.csv
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_instep_sw -o run -- python bench.py --dtype bf16sw --steps 5 --warmup 2 --no-cpu-baseline --no-north-star > gpurun_out/r06_instep_sw.log 2>&1 || { tail -30 gpurun_out/r06_instep_sw.log; exit 1; }
  python tools/prof_summary.py gpurun_out/r06_instep_sw/run_kernel_stats.csv 8 14
  rm -f gpurun_out/r06_instep_sw/run_kernel_trace.csv
fi
