cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -q -k shards --timeout 120 --timeout-method thread > gpurun_out/shard_tests.log 2>&1 || { tail -30 gpurun_out/shard_tests.log; exit 1; }
tail -2 gpurun_out/shard_tests.log
ANR_BENCH_BACKEND=gloo ANR_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --shard-frame --no-exact --steps 3 --warmup 1 > gpurun_out/shard_bench2.log 2>&1 || { tail -30 gpurun_out/shard_bench2.log; exit 1; }
tail -n 1 gpurun_out/shard_bench2.log | cut -c1-400
timeout -k 10 300 python bench.py --shard-frame --no-exact --no-cpu --steps 3 --warmup 1 > gpurun_out/shard_bench1.log 2>&1 || exit 1
tail -n 1 gpurun_out/shard_bench1.log | cut -c1-300
