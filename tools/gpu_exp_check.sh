# parity of experiment libraries (render tests, both precisions), then timing of the variants
# usage: tools/gpu_exp_check.sh "chk1 chk2" variant...
set -o pipefail
cd $GRAFT_REPO_ROOT
for CHK in $1; do
  ANR_LIB_PATH=animatable_nerf_amd/exp/$CHK.so timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 180 --timeout-method thread > gpurun_out/exp_${CHK}_tests.log 2>&1 || { tail -30 gpurun_out/exp_${CHK}_tests.log; exit 1; }
  echo "$CHK $(tail -1 gpurun_out/exp_${CHK}_tests.log)"
done
shift
bash tools/run_exp.sh "$@"
