# training parity + step time (both precisions) + kernel stats
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_anim.py -x -q --timeout 180 --timeout-method thread > gpurun_out/tr_tests.log 2>&1 || { tail -30 gpurun_out/tr_tests.log; exit 1; }
tail -2 gpurun_out/tr_tests.log
for p in bf16 fp32; do
  timeout -k 10 200 python bench.py --mode train --precision $p --no-cpu --steps 20 --warmup 3 > gpurun_out/tr_bench_$p.log 2>&1 || exit 1
  tail -n 1 gpurun_out/tr_bench_$p.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["precision"] if "precision" in d["config"] else "", d["ms_per_step"], d["value"])'
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof2_bf16 -o run --output-format csv -- python bench.py --mode train --precision bf16 --no-cpu --steps 20 --warmup 3 > gpurun_out/tprof2_bf16.log 2>&1 && echo prof_ok
