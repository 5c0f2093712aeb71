#!/bin/bash
# One C4 bench step with ATZ_TIMING=1 (host phase timings + per-level trial cycle breakdown).
# usage: tools/timing_run.sh <tag> [extra bench args]
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
ATZ_TIMING=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu "$@" > $O/timing.json 2> $O/timing.err
