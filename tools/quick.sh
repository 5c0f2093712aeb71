#!/bin/bash
# One GPU call for a kernel change: the -m gpu parity suite of tests/test_gpu.py, then a C4 bench
# line (3 steps, no CPU baseline).  usage: tools/quick.sh <tag> [bench args...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-quick}; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1 || exit 2
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000)" > $O/gen.log 2>&1 || exit 3
ATZ_TIMING=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h "$@" > $O/bench.json 2> $O/bench.err || exit 4
echo done
