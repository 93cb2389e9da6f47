set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mode sdf --no-cpu --no-exact --steps 5 --warmup 1 > gpurun_out/ab_nt1.log 2>&1 || exit 1
ANR_LIB_PATH=$PWD/ab/lib_nt0.so timeout -k 10 300 python bench.py --mode sdf --no-cpu --no-exact --steps 5 --warmup 1 > gpurun_out/ab_nt0.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode sdf --no-cpu --no-exact --steps 5 --warmup 1 > gpurun_out/ab_nt1b.log 2>&1 || exit 1
for f in ab_nt1 ab_nt0 ab_nt1b; do echo $f $(tail -1 gpurun_out/$f.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])"); done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k sdf > gpurun_out/ab_sdf_tests.log 2>&1 || { tail -30 gpurun_out/ab_sdf_tests.log; exit 1; }
tail -1 gpurun_out/ab_sdf_tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r3t2_prof -o run --output-format csv -- python bench.py --no-cpu --no-torch-baseline --no-host-render --steps 5 --warmup 2 > gpurun_out/r3t2_prof.log 2>&1 || exit 1
echo PROF_OK
