#!/bin/bash
# SQ instruction-mix counters per kernel on a C4 slice (two separate passes).  usage: tools/pmc_sq.sh <tag> [streams]
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; N=${2:-20000}
O=gpurun_out/$TAG; mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $O/p1 -o p --output-format csv -- python3 bench.py --streams $N --steps 1 --warmup 0 --no-cpu > $O/p1.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INSTS_VMEM -d $O/p2 -o p --output-format csv -- python3 bench.py --streams $N --steps 1 --warmup 0 --no-cpu > $O/p2.log 2>&1 || exit 2
