# sdf path check after a front-end change: sdf GPU tests, sdf bench, kernel stats of the sdf bench
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-knn}
timeout -k 10 400 python -u -m pytest tests/test_gpu_sdf.py -x -q --timeout 180 --timeout-method thread > gpurun_out/${T}_sdf_tests.log 2>&1 || { tail -40 gpurun_out/${T}_sdf_tests.log; exit 1; }
tail -1 gpurun_out/${T}_sdf_tests.log
timeout -k 10 300 python bench.py --mode sdf > gpurun_out/${T}_bench_sdf.log 2>&1 && tail -n 1 gpurun_out/${T}_bench_sdf.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_sdf_prof -o run --output-format csv -- python bench.py --mode sdf --no-cpu --steps 2 --warmup 1 > gpurun_out/${T}_sdf_prof.log 2>&1 && echo PROF_OK
