#!/bin/bash
# round pass: GPU tests, default bench + rocprof stats, f32 bench line, host enqueue time
set -o pipefail
bash tools/gpu_round.sh r03q || exit 1
echo "-- f32"
timeout -k 10 400 python -u bench.py --dtype f32 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r03q_bench_f32.json 2> gpurun_out/r03q_bench_f32.err || { tail -20 gpurun_out/r03q_bench_f32.err; exit 1; }
cut -c1-400 gpurun_out/r03q_bench_f32.json
echo "-- host enqueue"
timeout -k 10 300 python -u tools/host_time.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03q_host_time.txt
