#!/bin/bash
# Interleaved A/B of environment settings on the C4 bench (one JSON line per run).
# usage: tools/ab_env.sh <tag> <reps> "<env settings A>" "<env settings B>" ...   ("-" = no settings)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'.')
from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000)" || exit 1
for ((i=1;i<=R;i++)); do
  k=0
  for E in "$@"; do
    k=$((k+1))
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/$TAG/v$k.$i.json 2> gpurun_out/$TAG/v$k.$i.err || exit 1
    echo "v$k.$i [$E] $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG/v$k.$i.json'));print(d['value'],(d['reconstruct'] or {}).get('atz_sha256'),{x:d['detail'].get(x) for x in ('k_trial_ms','k_match_ms','k_chains_ms','k_inflate_ms','n_trials','n_trials_replayed','n_replay_checked','n_trials_duplicate')})")"
  done
done
