#!/bin/bash
# Throughput ceiling from concurrency: 1, 2 and 3 independent C4 files in flight on one GPU (one context
# and host thread each, bench.py --mode shards --files-per-gpu k), then a rocprofv3 kernel trace of one
# 12 500-stream step.  usage: tools/ceiling.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ceiling}; mkdir -p $O
timeout -k 10 400 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen
for s in (4, 5, 6): datagen.cached('c4','/tmp/atz_bench_cache',seed=s,n_streams=100000)
datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500)" > $O/gen.log 2>&1 || exit 3
for k in 1 2 3; do
  timeout -k 10 300 python3 bench.py --mode shards --files-per-gpu $k --steps 2 --warmup 1 --no-cpu --no-h2h --no-recon > $O/f$k.json 2> $O/f$k.err || exit 4
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o p --output-format csv -- python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/tr.json 2> $O/tr.err || exit 5
echo done
