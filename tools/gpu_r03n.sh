#!/bin/bash
# deterministic vs atomic reductions, same box, alternating
set -o pipefail
for i in 1 2; do
echo "-- deterministic"
timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
echo "-- atomic"
NRSE_ATOMIC_REDUCTIONS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
timeout -k 10 200 python -u tools/bench_gemm_fwd.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/bench_gemm_bwd.py 2>&1 | grep -v amdgpu.ids
