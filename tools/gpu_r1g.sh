set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1g_gpu_tests.log 2>&1 && tail -3 gpurun_out/r1g_gpu_tests.log && \
timeout -k 10 300 python bench.py > gpurun_out/r1g_bench.log 2>&1 && tail -c 400 gpurun_out/r1g_bench.log && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r1g_prof -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r1g_prof.log 2>&1 && echo PROF_OK
