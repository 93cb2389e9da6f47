cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sdfprof -o run --output-format csv -- python bench.py --mode sdf --render-precision bf16x3 --no-cpu --steps 2 --warmup 1 > gpurun_out/sdfprof.log 2>&1 && echo ok
