#!/bin/bash
# Trials in flight over the sweep (ATZ_TIMING=3: per-trial s_memrealtime spans): the 12 500-stream share
# with 3 pipes and with 6 pipes on 8 hardware queues (the N = 8 configuration), and the full C4.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-inflight}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || exit 2
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000); datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500)" > $O/gen.log 2>&1 || exit 3
ATZ_TIMING=3 timeout -k 10 300 python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/s3.json 2> $O/s3.err || exit 4
ATZ_TIMING=3 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/s6.json 2> $O/s6.err || exit 5
ATZ_TIMING=3 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/full.json 2> $O/full.err || exit 6
echo done
