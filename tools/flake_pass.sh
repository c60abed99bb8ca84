#!/bin/bash
# Run the GPU test suite N times (numeric flake hunt; no -x); stops at anything but pass/fail.
N=${1:-3}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:warnings > gpurun_out/flake_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $(tail -1 gpurun_out/flake_$i.log)"
  grep -E "^FAILED" gpurun_out/flake_$i.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
