#!/bin/bash
# One GPU call: tests/test_gpu.py parity suite, a C4 bench line (3 steps, no CPU baseline), then the
# ATZ_TIMING=2 sweep timelines of one full C4 step and of a 12 500-stream file (one rank's share at
# 8 GPUs).  usage: tools/probe.sh <tag> [notest]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-probe}
O=gpurun_out/$TAG; mkdir -p $O
if [ "$2" != notest ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1 || exit 2
fi
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000); datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500)" > $O/gen.log 2>&1 || exit 3
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-h2h > $O/bench.json 2> $O/bench.err || exit 4
ATZ_TIMING=2 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-h2h > $O/timing.json 2> $O/timing.err || exit 5
ATZ_TIMING=2 timeout -k 10 200 python3 bench.py --streams 12500 --steps 2 --warmup 1 --no-cpu --no-h2h > $O/small.json 2> $O/small.err || exit 6
echo done
