#!/bin/bash
# Interleaved A/B of environment settings on the C4 bench (one JSON line per run).
# usage: tools/ab_env.sh <tag> <reps> "<env settings A>" "<env settings B>" ...   ("-" = no settings)
# AB_STREAMS=n: a file of n streams instead of the full C4 (e.g. 12500, one rank's share at 8 GPUs)
# AB_WORKLOAD=c2|c3|c5: another BASELINE config (bench.py --workload)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'.')
from antiz_amd import datagen
w='${AB_WORKLOAD:-c4}'
datagen.cached(w,'/tmp/atz_bench_cache',**({} if w in ('c2','c3') else dict(seed=5 if w=='c5' else 4,n_streams=${AB_STREAMS:-100000})))" || exit 1
for ((i=1;i<=R;i++)); do
  k=0
  for E in "$@"; do
    k=$((k+1))
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 240 python3 bench.py --workload ${AB_WORKLOAD:-c4} --streams ${AB_STREAMS:-100000} --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h > gpurun_out/$TAG/v$k.$i.json 2> gpurun_out/$TAG/v$k.$i.err || exit 1
    echo "v$k.$i [$E] $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG/v$k.$i.json'));print(d['value'],d['ms_per_step'],(d.get('atz_parity') or {}).get('identical_to_reference'),{x:d['detail'].get(x) for x in ('k_trial_ms','k_match_ms','k_chains_ms','k_inflate_ms','n_trials','n_trials_replayed','n_replay_checked','n_trials_duplicate','n_trials_speculative','n_trials_skipped')})")"
  done
done
