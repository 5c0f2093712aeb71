#!/bin/bash
# A/B of environment settings on the C4 bench: tools/exp_env.sh <tag> "ENV=.. ENV2=.." "ENV=.." ...
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 240 python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/$TAG/v$i.json 2> gpurun_out/$TAG/v$i.err || exit 1
  echo "$E" > gpurun_out/$TAG/v$i.env
done
