cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python bench.py --steps 1 --warmup 0 --no-cpu --no-exact"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o l2 --output-format csv -- $B > gpurun_out/pmc_l2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_sq -o sq --output-format csv -- $B > gpurun_out/pmc_sq.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum -d gpurun_out/pmc_tcp -o tcp --output-format csv -- $B > gpurun_out/pmc_tcp.log 2>&1
