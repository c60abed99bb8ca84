#!/bin/bash
# rocprofv3 kernel trace of the train_byol CLI on the dev YAML (configs[0] shape, mock pairs), then
# the non-library dispatches between its training steps (tools/trace_train_loop.py).
# Usage (on the GPU box): bash tools/trace_train_loop.sh TAG
set -o pipefail
TAG=${1:-r06_trainloop}
mkdir -p gpurun_out
RUN=$(mktemp -d /tmp/trainloop.XXXX)   # checkpoints land here, not under gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CONF=$GRAFT_REPO_ROOT/tests/golden/configs/dev_wavlm-large_byol.yaml
OUT=$GRAFT_REPO_ROOT/gpurun_out
(cd $RUN && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$TAG -o run -- \
  python $GRAFT_REPO_ROOT/noise-robust-speech-embedding_amd/train_byol.py --config $CONF --device cuda:0 \
  --batch_size 4 --epochs 1 --mock_items 96 --max_steps 16 > $OUT/$TAG.log 2>&1) || { tail -30 $OUT/$TAG.log; exit 1; }
grep -E "Epoch|complete" $OUT/$TAG.log
python tools/trace_train_loop.py $OUT/$TAG/run_kernel_trace.csv 16 | tee $OUT/$TAG.txt
rm -rf $RUN $OUT/$TAG/run_kernel_trace.csv
