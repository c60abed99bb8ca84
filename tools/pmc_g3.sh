set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=noise-robust-speech-embedding_amd/build/diag
NRSE_LIB_PATH=$D/libnrse_diag1.so timeout -k 10 120 python tools/diag_g3.py
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc1 -o run -- python tools/diag_g3.py > gpurun_out/pmc1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc2 -o run -- python tools/diag_g3.py > gpurun_out/pmc2.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc3 -o run -- python tools/diag_g3.py > gpurun_out/pmc3.log 2>&1
ls gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3
