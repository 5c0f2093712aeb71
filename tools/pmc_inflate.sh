export TMPDIR=/tmp
export EXP_N=4000
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/pmc1 -o p --output-format csv -- python3 tools/exp_inflate.py > gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC -d gpurun_out/pmc2 -o p --output-format csv -- python3 tools/exp_inflate.py > gpurun_out/pmc2.log 2>&1
