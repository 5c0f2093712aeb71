#!/bin/bash
# Interleaved A/B of library builds on the C4 bench: tools/ab.sh <tag> <reps> lib1 lib2 ...
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out/$TAG
for ((i=1;i<=R;i++)); do
  for L in "$@"; do
    n=$(basename $L .so)
    ATZ_LIB=$L timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/$TAG/$n.$i.json 2> gpurun_out/$TAG/$n.$i.err || exit 1
  done
done
