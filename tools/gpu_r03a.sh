#!/bin/bash
# r03 first pass: the new parity tests (RCCL, Large 3/8/12 s, f32 attention T>400, bf16 vs oracle at
# 8/12 s, optimizer state / early stop), then the self-launching 2-rank bench (gloo, shared device).
set -o pipefail
TAG=${1:-r03a}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_model_gpu.py::test_optimizer_state_roundtrip_resumes tests/test_attention_gpu.py \
  tests/test_large_gpu.py tests/test_bf16_gpu.py -x -v -s --timeout 400 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|large_|f32_|bf16_" gpurun_out/${TAG}_tests.log | tail -70
[ $rc -eq 0 ] || exit $rc
NRSE_SHARE_DEVICE=1 NRSE_DDP_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --batch 8 \
  > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err || { tail -30 gpurun_out/${TAG}_bench2.err; exit 1; }
cat gpurun_out/${TAG}_bench2.json
