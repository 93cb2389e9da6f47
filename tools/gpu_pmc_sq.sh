# SQ instruction-mix / stall counters of the fused render kernel (one --pmc pass each)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r2b}
B="python bench.py --steps 1 --warmup 0 --no-cpu --no-exact"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex k_mlp_b16 -d gpurun_out/${T}_pmc1 -o p --output-format csv -- $B > gpurun_out/${T}_pmc1.log 2>&1 && echo P1_OK && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA --kernel-include-regex k_mlp_b16 -d gpurun_out/${T}_pmc2 -o p --output-format csv -- $B > gpurun_out/${T}_pmc2.log 2>&1 && echo P2_OK
