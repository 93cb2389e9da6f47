# same-box A/B of the sdf render's batch size (ab/lib_b*.so built with -DANR_SDF_BATCH_LOG2=N)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --mode sdf --no-cpu --no-exact --steps 5 --warmup 1"
timeout -k 10 300 $B > gpurun_out/abb_19.log 2>&1 || exit 1
ANR_LIB_PATH=$PWD/ab/lib_b20.so timeout -k 10 300 $B > gpurun_out/abb_20.log 2>&1 || exit 1
ANR_LIB_PATH=$PWD/ab/lib_b21.so timeout -k 10 300 $B > gpurun_out/abb_21.log 2>&1 || exit 1
timeout -k 10 300 $B > gpurun_out/abb_19b.log 2>&1 || exit 1
for f in abb_19 abb_20 abb_21 abb_19b; do echo $f $(tail -1 gpurun_out/$f.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])"); done
