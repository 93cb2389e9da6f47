# HBM traffic of the fused render kernel: FETCH_SIZE and WRITE_SIZE in separate --pmc passes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python bench.py --steps 1 --warmup 0 --no-cpu --no-exact"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o f --output-format csv -- $B > gpurun_out/pmc_f.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o w --output-format csv -- $B > gpurun_out/pmc_w.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o l2 --output-format csv -- $B > gpurun_out/pmc_l2.log 2>&1 && echo PMC_OK
