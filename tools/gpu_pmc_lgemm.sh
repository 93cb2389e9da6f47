# SQ / L2 counters of the sdf layer GEMMs (k_lgemm), one --pmc pass each, one sdf frame
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-lg}
B="python bench.py --mode sdf --steps 1 --warmup 0 --no-cpu"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex k_lgemm -d gpurun_out/${T}_pmc1 -o p --output-format csv -- $B > gpurun_out/${T}_pmc1.log 2>&1 && echo P1_OK && \
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT --kernel-include-regex k_lgemm -d gpurun_out/${T}_pmc2 -o p --output-format csv -- $B > gpurun_out/${T}_pmc2.log 2>&1 && echo P2_OK && \
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_lgemm -d gpurun_out/${T}_pmc3 -o p --output-format csv -- $B > gpurun_out/${T}_pmc3.log 2>&1 && echo P3_OK && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_lgemm -d gpurun_out/${T}_pmc4 -o p --output-format csv -- $B > gpurun_out/${T}_pmc4.log 2>&1 && echo P4_OK && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_lgemm -d gpurun_out/${T}_pmc5 -o p --output-format csv -- $B > gpurun_out/${T}_pmc5.log 2>&1 && echo P5_OK
