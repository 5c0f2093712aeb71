#!/bin/bash
# Round-4 measurement call: every GPU step under its own time limit, the chain stops at the first failure.
# usage: tools/measure.sh <tag> [stages...]
#   stages: test (whole -m gpu suite), gpu (tests/test_gpu.py + knobs), bench (the driver's default command),
#           prof (rocprofv3 kernel trace + stats of one step), sq (two SQ counter passes + GRBM_GUI_ACTIVE),
#           pmc (FETCH_SIZE and WRITE_SIZE passes), small (12 500-stream share, ATZ_TIMING=2),
#           timing (ATZ_TIMING=2 full step)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-m}; shift
STAGES=${*:-"gpu bench prof"}
O=gpurun_out/$TAG; mkdir -p $O
has() { [[ " $STAGES " == *" $1 "* ]]; }
B1="bench.py --steps 1 --warmup 0 --no-cpu --no-recon --no-h2h"
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'.')
from antiz_amd import datagen; print(datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000)); print(datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500))" > $O/gen.log 2>&1 || exit 1
if has test; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1 || exit 2
fi
if has gpu; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_knobs.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1 || exit 2
fi
if has bench; then
  timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 3
fi
if has timing; then
  ATZ_TIMING=2 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/timing.json 2> $O/timing.err || exit 7
fi
if has small; then
  ATZ_TIMING=2 timeout -k 10 200 python3 bench.py --streams 12500 --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h > $O/small.json 2> $O/small.err || exit 8
fi
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 $B1 > $O/prof.json 2> $O/prof.err || exit 4
fi
if has sq; then
  timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $O/sq1 -o p --output-format csv -- python3 $B1 > $O/sq1.json 2> $O/sq1.err || exit 5
  timeout -s KILL 400 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d $O/sq2 -o p --output-format csv -- python3 $B1 > $O/sq2.json 2> $O/sq2.err || exit 6
fi
if has pmc; then
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf -o p --output-format csv -- python3 $B1 > $O/pmcf.json 2> $O/pmcf.err || exit 9
  timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw -o p --output-format csv -- python3 $B1 > $O/pmcw.json 2> $O/pmcw.err || exit 10
fi
echo done
