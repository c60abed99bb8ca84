#!/bin/bash
# Roofline evidence for bench.py's line: the default bench (with its serialised
# GEMM probe step), a rocprofv3 kernel-trace of the same bench with the streams serialised
# (NRSE_SERIAL_TARGET=1: per-kernel durations without concurrent-stream sharing), and the PMC
# traffic passes. Usage: bash tools/gpu_roofline.sh TAG
set -o pipefail
TAG=${1:-roof}
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NRSE_SERIAL_TARGET=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_serial -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_serial.log 2>&1 || { tail -30 gpurun_out/${TAG}_serial.log; exit 1; }
grep '"metric"' gpurun_out/${TAG}_serial.log | cut -c1-200
python tools/prof_summary.py gpurun_out/${TAG}_serial/run_kernel_stats.csv 8 12
bash tools/pmc_gemm.sh ${TAG}
