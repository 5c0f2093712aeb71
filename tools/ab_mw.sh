#!/bin/bash
# Interleaved A/B of environment settings on the full C4 bench and the 12 500-stream file.
# usage: tools/ab_mw.sh <tag> <reps> "<env A>" "<env B>" ...   ("-" = no settings)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for ((i=1;i<=R;i++)); do
  k=0
  for E in "$@"; do
    k=$((k+1)); [ "$E" = "-" ] && E=""
    env $E timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h > $O/full_v$k.$i.json 2> $O/full_v$k.$i.err || exit 1
    env $E timeout -k 10 240 python3 bench.py --streams 12500 --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h > $O/small_v$k.$i.json 2> $O/small_v$k.$i.err || exit 2
  done
done
echo done
