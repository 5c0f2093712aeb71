#!/bin/bash
# Exclusive kernel times (one sweep pipe, nothing overlaps) and the default 3-pipe step, both with
# ATZ_TIMING=1 host-phase timings.  usage: tools/breakdown.sh <tag>
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'.')
from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000)" > $O/gen.log 2>&1 || exit 1
ATZ_PIPES=1 ATZ_TIMING=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/p1.json 2> $O/p1.err || exit 2
ATZ_TIMING=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/p3.json 2> $O/p3.err || exit 3
echo done
