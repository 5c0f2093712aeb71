#!/bin/bash
# Round-5 diagnostics: per-round trial completion quantiles and the round timeline (ATZ_TIMING=3) on the
# 12 500-stream share with six pipes on eight hardware queues (one rank at N = 8) and on the full C4.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-diag}; mkdir -p $O
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000); datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500)" > $O/gen.log 2>&1 || exit 3
ATZ_TIMING=3 ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/s6.json 2> $O/s6.err || exit 4
ATZ_TIMING=3 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/full.json 2> $O/full.err || exit 6
echo done
