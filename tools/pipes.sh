#!/bin/bash
# 12 500-stream share under 3 / 6 / 12 pipes (4 / 8 / 16 hardware queues), ATZ_TIMING=3: trials in flight,
# time in HIP copy calls and syncs per pipe.  usage: tools/pipes.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pipes}; mkdir -p $O
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500)" > $O/gen.log 2>&1 || exit 3
ATZ_TIMING=3 timeout -k 10 300 python3 bench.py --streams 12500 --steps 2 --warmup 1 --no-cpu --no-recon --no-h2h > $O/p3.json 2> $O/p3.err || exit 4
ATZ_TIMING=3 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --streams 12500 --steps 2 --warmup 1 --no-cpu --no-recon --no-h2h > $O/p6.json 2> $O/p6.err || exit 5
ATZ_TIMING=3 GPU_MAX_HW_QUEUES=16 ATZ_PIPES=8 timeout -k 10 300 python3 bench.py --streams 12500 --steps 2 --warmup 1 --no-cpu --no-recon --no-h2h > $O/p8.json 2> $O/p8.err || exit 6
echo done
