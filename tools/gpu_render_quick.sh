# render parity with the in-tree library, then timing of variants (base = in-tree library)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_mesh.py -x -q --timeout 180 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 || { tail -30 gpurun_out/quick_tests.log; exit 1; }
tail -1 gpurun_out/quick_tests.log
bash tools/run_exp.sh "$@"
