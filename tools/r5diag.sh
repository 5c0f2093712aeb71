#!/bin/bash
# Round-5 diagnostics: per-round trial completion quantiles and the round timeline (ATZ_TIMING=3) on the
# 12 500-stream share with six pipes on eight hardware queues (one rank at N = 8) and on the full C4,
# each with the extra environment given (e.g. "ATZ_PRERUN=8").  usage: tools/r5diag.sh <tag> [env...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-diag}; shift; mkdir -p $O
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000); datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500)" > $O/gen.log 2>&1 || exit 3
k=0
for E in "$@"; do
  k=$((k+1)); [ "$E" = "-" ] && E=""
  env $E ATZ_TIMING=3 ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/s6_$k.json 2> $O/s6_$k.err || exit 4
  env $E ATZ_TIMING=3 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/full_$k.json 2> $O/full_$k.err || exit 6
done
echo done
