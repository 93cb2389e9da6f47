# kernel trace of the training bench (per-dispatch durations, grids, gaps)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-tr}
timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 3 > gpurun_out/${T}_bench_train.log 2>&1 || { tail -20 gpurun_out/${T}_bench_train.log; exit 1; }
tail -n 1 gpurun_out/${T}_bench_train.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_trace -o run --output-format csv -- python bench.py --mode train --steps 3 --warmup 2 > gpurun_out/${T}_trace.log 2>&1 && echo TRACE_OK
