#!/bin/bash
# Per-kernel picture of the current tree: isolated attention / forward-GEMM microbenches, the
# default bench with per-shape GEMM detail, and rocprofv3 kernel-trace stats of the bench with the
# streams serialised. Usage (on the GPU box): bash tools/gpu_prof.sh TAG
set -o pipefail
TAG=${1:-prof}
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/${TAG}_attn.txt 2>&1 || { tail -20 gpurun_out/${TAG}_attn.txt; exit 1; }
cat gpurun_out/${TAG}_attn.txt
timeout -k 10 180 python -u tools/bench_gemm_fwd.py > gpurun_out/${TAG}_gemm_fwd.txt 2>&1 || { tail -20 gpurun_out/${TAG}_gemm_fwd.txt; exit 1; }
cat gpurun_out/${TAG}_gemm_fwd.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --detail gpurun_out/${TAG}_detail.json > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NRSE_SERIAL_TARGET=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_serial -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_serial.log 2>&1 || { tail -30 gpurun_out/${TAG}_serial.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_serial/run_kernel_stats.csv 9 30
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_instep -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_instep.log 2>&1 || { tail -30 gpurun_out/${TAG}_instep.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_instep/run_kernel_stats.csv 9 30
