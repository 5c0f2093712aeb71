#!/bin/bash
# 12 500-stream share: more pipes with the speculation depth of 3 (ATZ_KREF=3), on 8 / 16 / 24 hardware
# queues, ATZ_TIMING=3 (trials in flight).  usage: tools/pipes2.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pipes2}; mkdir -p $O
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500); datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000)" > $O/gen.log 2>&1 || exit 3
run() { local tag=$1; shift; env "$@" ATZ_TIMING=3 timeout -k 10 300 python3 bench.py --streams 12500 --steps 2 --warmup 1 --no-cpu --no-recon --no-h2h > $O/$tag.json 2> $O/$tag.err || exit 4; }
run k3p3 ATZ_KREF=3
run k3p6 ATZ_KREF=3 ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8
run k3p8 ATZ_KREF=3 ATZ_PIPES=8 GPU_MAX_HW_QUEUES=16
run k3p8q32 ATZ_KREF=3 ATZ_PIPES=8 GPU_MAX_HW_QUEUES=32
ATZ_KREF=3 ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-recon --no-h2h > $O/full_k3p6.json 2> $O/full_k3p6.err || exit 5
echo done
