cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_sdf.py -x -v --timeout 180 --timeout-method thread > gpurun_out/sdf_tests.log 2>&1 || { tail -40 gpurun_out/sdf_tests.log; exit 1; }
tail -3 gpurun_out/sdf_tests.log
for p in bf16x3 fp32; do
  timeout -k 10 300 python bench.py --mode sdf --render-precision $p --no-cpu --steps 3 --warmup 1 > gpurun_out/sdf_bench_$p.log 2>&1 || exit 1
  echo $p $(tail -n 1 gpurun_out/sdf_bench_$p.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["frac"])')
done
