# training step profile (bf16 and fp32): kernel stats per precision
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for p in bf16 fp32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof_$p -o run --output-format csv -- python bench.py --mode train --precision $p --no-cpu --steps 20 --warmup 3 > gpurun_out/tprof_$p.log 2>&1 || exit 1
done
echo done
