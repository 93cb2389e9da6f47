# time the training step (bf16) with experiment libraries: tools/gpu_train_exp.sh name...
cd $GRAFT_REPO_ROOT
for n in "$@"; do
  if [ "$n" = base ]; then lib=""; else lib=animatable_nerf_amd/exp/$n.so; fi
  ANR_LIB_PATH=$lib timeout -k 10 200 python bench.py --mode train --precision bf16 --no-cpu --steps 20 --warmup 3 > gpurun_out/texp_$n.log 2>&1 || exit 1
  echo "$n $(tail -n 1 gpurun_out/texp_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
ANR_LIB_PATH=animatable_nerf_amd/exp/bk128.so timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 180 --timeout-method thread > gpurun_out/texp_tests.log 2>&1; tail -1 gpurun_out/texp_tests.log
