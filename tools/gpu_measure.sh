#!/bin/bash
# One GPU call: parity suite, default bench line (with CPU baseline), rocprofv3 kernel stats of one
# step, and separate PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic.  Every GPU step has its
# own time limit; the chain stops at the first failure.
# usage: tools/gpu_measure.sh <tag> [stages...]
#   stages: test bench prof pmc timing small shardtest file2 file4 grid knobs c2 c3 c5 (default: test bench prof pmc)
#   timing: ATZ_TIMING=2 timeline of one C4 step; small: the same on a 12 500-stream file (one rank's
#   share of C4 at 8 GPUs); shardtest: the one-file multi-rank tests only; fileN: bench.py --gpus N on one
#   1 GB file with N ranks sharing the box's GPU over gloo (rehearsal of the driver's RCCL run)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}; shift
STAGES=${*:-"test bench prof pmc"}
O=gpurun_out/$TAG; mkdir -p $O
has() { [[ " $STAGES " == *" $1 "* ]]; }
# workload generated once, before any timed/profiled run
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'.')
from antiz_amd import datagen; print(datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000))" > $O/gen.log 2>&1 || exit 1
if has test; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1 || exit 2
fi
if has grid; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_grid.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/grid.log 2>&1 || exit 11
fi
if has knobs; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_knobs.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/knobs.log 2>&1 || exit 12
fi
for W in c2 c3 c5; do
  if has $W; then
    timeout -k 10 600 python3 bench.py --workload $W > $O/$W.json 2> $O/$W.err || exit 13
  fi
done
if has bench; then
  timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 3
fi
if has timing; then
  ATZ_TIMING=2 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon > $O/timing.json 2> $O/timing.err || exit 7
fi
if has small; then
  ATZ_TIMING=2 timeout -k 10 200 python3 bench.py --streams 12500 --steps 2 --warmup 1 --no-cpu --no-recon > $O/small.json 2> $O/small.err || exit 8
fi
if has shardtest; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_shard.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/shardtest.log 2>&1 || exit 9
fi
for N in 2 4 8; do
  if has file$N; then
    ATZ_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 2 --warmup 1 --no-recon > $O/file$N.json 2> $O/file$N.err || exit 10
  fi
done
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-recon --no-h2h > $O/prof.json 2> $O/prof.err || exit 4
fi
if has pmc; then
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-recon --no-h2h > $O/pmcf.json 2> $O/pmcf.err || exit 5
  timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-recon --no-h2h > $O/pmcw.json 2> $O/pmcw.err || exit 6
fi
echo done
