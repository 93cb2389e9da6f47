# sdf split-bf16 layer GEMM: parity (sdf GPU tests), frame bench, per-kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_sdf.py -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/lg_tests.log 2>&1 || { tail -40 gpurun_out/lg_tests.log; exit 1; }
tail -3 gpurun_out/lg_tests.log
timeout -k 10 300 python bench.py --mode sdf --no-cpu > gpurun_out/lg_bench_sdf.log 2>&1 || { tail -20 gpurun_out/lg_bench_sdf.log; exit 1; }
tail -n 1 gpurun_out/lg_bench_sdf.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lg_prof -o run --output-format csv -- python bench.py --mode sdf --no-cpu --steps 2 --warmup 1 > gpurun_out/lg_prof.log 2>&1 && echo PROF_OK
B="python bench.py --mode sdf --steps 1 --warmup 0 --no-cpu"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/lg_pmc_f -o f --output-format csv -- $B > gpurun_out/lg_pmc_f.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/lg_pmc_w -o w --output-format csv -- $B > gpurun_out/lg_pmc_w.log 2>&1 && echo PMC_OK
