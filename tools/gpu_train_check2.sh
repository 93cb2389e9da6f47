# training parity (GPU) + training bench
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-trc}
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_anim.py -x -q --timeout 180 --timeout-method thread > gpurun_out/${T}_train_tests.log 2>&1 || { tail -40 gpurun_out/${T}_train_tests.log; exit 1; }
tail -1 gpurun_out/${T}_train_tests.log
for prec in bf16 fp32; do
timeout -k 10 300 python bench.py --mode train --precision $prec --steps 10 --warmup 3 > gpurun_out/${T}_bench_train_$prec.log 2>&1 || { tail -20 gpurun_out/${T}_bench_train_$prec.log; exit 1; }
tail -n 1 gpurun_out/${T}_bench_train_$prec.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["dtype"], d["value"], d["ms_per_step"], d["loss_last_step"])'
done
