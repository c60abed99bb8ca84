set -o pipefail
TAG=r02_v10
timeout -k 10 300 python -u tools/diag_dropin.py 5 > gpurun_out/diag_dropin.log 2>&1 || { tail -20 gpurun_out/diag_dropin.log; exit 1; }
grep rep gpurun_out/diag_dropin.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_profbench.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/${TAG}_profbench.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_prof/run_kernel_stats.csv 7 12
