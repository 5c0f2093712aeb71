#!/bin/bash
# 12 500-stream share: speculation depth (ATZ_TARGET) and extra trial LDS (ATZ_XLDS), trials in flight
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-spec}; mkdir -p $O
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500); datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000)" > $O/gen.log 2>&1 || exit 3
run() { local tag=$1; shift; env "$@" ATZ_TIMING=3 timeout -k 10 300 python3 bench.py --streams 12500 --steps 2 --warmup 1 --no-cpu --no-recon --no-h2h > $O/$tag.json 2> $O/$tag.err || exit 4; }
run base ATZ_TARGET=4096
run t8k ATZ_TARGET=8192
run t16k ATZ_TARGET=16384
run x24k ATZ_XLDS=24576
ATZ_XLDS=24576 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-recon --no-h2h > $O/full_x24k.json 2> $O/full_x24k.err || exit 5
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-recon --no-h2h > $O/full_base.json 2> $O/full_base.err || exit 5
echo done
