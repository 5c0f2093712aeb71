#!/bin/bash
# A/B of library builds on the C4 bench (2 timed steps each): tools/exp_variants.sh <tag> lib1 lib2 ...
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for L in "$@"; do
  n=$(basename $L .so)
  ATZ_LIB=$L timeout -k 10 240 python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/$TAG/$n.json 2> gpurun_out/$TAG/$n.err || exit 1
done
