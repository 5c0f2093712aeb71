#!/bin/bash
# Host CPU profile of the sweep (ATZ_HOSTPROF sampling inside libatz_accel): the full C4 run and the
# 12 500-stream share on six pipes, one timed step each.  Resolve here with tools/hostprof.py.
# usage: tools/hostprof.sh <tag> [env...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-hp}; shift; mkdir -p $O; rm -f $O/*.prof
E="$*"; [ "$E" = "-" ] && E=""
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000); datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500)" > $O/gen.log 2>&1 || exit 3
env $E ATZ_HOSTPROF=$O/full.prof timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/full.json 2> $O/full.err || exit 4
env $E ATZ_HOSTPROF=$O/s6.prof ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/s6.json 2> $O/s6.err || exit 5
echo done
