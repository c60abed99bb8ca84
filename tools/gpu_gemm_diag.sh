#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
D=noise-robust-speech-embedding_amd/build/diag
timeout -k 10 120 python tools/diag_g3.py > gpurun_out/diag.log 2>&1 || { cat gpurun_out/diag.log; exit 1; }
for n in 1 2 3 4 5 6; do NRSE_LIB_PATH=$D/libnrse_diag$n.so timeout -k 10 120 python tools/diag_g3.py >> gpurun_out/diag.log 2>&1 || { tail gpurun_out/diag.log; exit 1; }; done
cat gpurun_out/diag.log
timeout -k 10 200 python tools/bench_gemm_epi.py 2>&1 | tee gpurun_out/epi.log
NRSE_SERIAL_TARGET=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --detail gpurun_out/detail_serial.json > gpurun_out/detail_serial.log 2>&1
python - <<'PY'
import json
d = json.load(open("gpurun_out/detail_serial.json"))
tot = sum(v["ms_total"] for v in d.values())
for k, v in list(d.items())[:24]:
    print(f"{k:32s} {v['ms_total']/5:7.2f} ms/step  {v['tflops']:6.0f} TF  n={v['launches']/5:.1f}")
print("total", tot / 5)
PY
